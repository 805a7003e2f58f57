// bre_oracle.cpp — CPU restatement of the reference photon-beam gather (TEST INFRASTRUCTURE).
//
// THIS FILE IS THE PARITY ORACLE AND THE CPU BASELINE, NOT THE PRODUCT.  Only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg may load the library built from it.
// The product path (libbre.so, HIP) never links, calls or falls back to this code.
//
// What it restates (reference = bwiberg/beam-radiance-estimate-pbrt, read as text only):
//   * PhotonBeam::WorldBound              src/core/photonbeambvh.h:60-72  (+ Bounds3 ctor geometry.h:759-763)
//   * Bounds3::IntersectP(ray,invDir,neg) src/core/geometry.h:1410-1436, gamma(3) src/core/pbrt.h:263-265
//   * Determinant / ComputeClosestPoints  src/integrators/photonbeam.cpp:79-186
//   * PhotonBeamBVH SAH build (12 buckets, maxPrimsInNode=1), DFS flatten, stack traversal
//                                         src/core/photonbeambvh.cpp:204-248, 259-425, 663-723
//   * gather + 1D kernel                  src/integrators/photonbeam.cpp:494-508
//   * radius schedule                     src/integrators/photonbeam.cpp:354-356, 562
//   * Union / Offset / Clamp semantics    src/core/geometry.h:801-807, 1250-1266; src/core/pbrt.h:278-284
//   * Cross in double                     src/core/geometry.h:957-963
//   * Vector3 operator/ (multiply by 1/f) src/core/geometry.h:244-257
//
// Parity status: UNPINNED for the gather path.  The reference's own tests contain no test,
// golden vector or fixture for photonbeam / photonbeambvh and building or
// running the reference in this environment was denied.  The restatement is
// checked instead against hand-derived known-answer tests and an independent pure-Python
// restatement (tests/test_oracle_kat.py, tests/test_oracle_crosscheck.py).
//
// Interpretation notes (where the C++ text admits two readings, the libstdc++/GCC one is used):
//   * WorldBound's unqualified `sqrt(1 - dir.x*dir.x)` resolves to ::sqrt(double) with
//     libstdc++ (<cmath> only; checked with this image's g++), so `2*radius*sqrt(..)` and the
//     following `+` are evaluated in double and rounded to float once (sqrt_mode=0).
//     sqrt_mode=1 selects the all-float reading.
//   * x86-64 SSE float arithmetic, no FMA contraction (-ffp-contract=off), IEEE division/sqrt.
//
// Build: oracle/Makefile  (g++ -O3 -ffp-contract=off -fno-fast-math).

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <memory>
#include <thread>
#include <vector>

namespace ora {

typedef float Float;

struct V3 {
    Float x, y, z;
    V3() : x(0), y(0), z(0) {}
    V3(Float a, Float b, Float c) : x(a), y(b), z(c) {}
    Float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
    Float &operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
};
static inline V3 add(V3 a, V3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V3 sub(V3 a, V3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
// Vector3::operator*(U s) -> (s*x, s*y, s*z)   geometry.h:231-233
static inline V3 mul(V3 a, Float s) { return V3(s * a.x, s * a.y, s * a.z); }
// Vector3::operator/(U f): inv = (Float)1/f; x*inv   geometry.h:244-248
static inline V3 divv(V3 a, Float f) {
    Float inv = (Float)1 / f;
    return V3(a.x * inv, a.y * inv, a.z * inv);
}
static inline Float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline Float lengthSq(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
static inline Float length(V3 a) { return std::sqrt(lengthSq(a)); }
// Cross in double, geometry.h:957-963
static inline V3 cross(V3 v1, V3 v2) {
    double v1x = v1.x, v1y = v1.y, v1z = v1.z;
    double v2x = v2.x, v2y = v2.y, v2z = v2.z;
    return V3((Float)((v1y * v2z) - (v1z * v2y)), (Float)((v1z * v2x) - (v1x * v2z)),
              (Float)((v1x * v2y) - (v1y * v2x)));
}
template <typename T, typename U, typename V>
static inline T Clamp(T val, U low, V high) {  // pbrt.h:278-284
    if (val < low) return low;
    else if (val > high) return high;
    else return val;
}
// std::min / std::max exactly (NaN behaviour matters): min(a,b) = (b<a)?b:a, max(a,b) = (a<b)?b:a
static inline Float smin(Float a, Float b) { return (b < a) ? b : a; }
static inline Float smax(Float a, Float b) { return (a < b) ? b : a; }

struct Box {
    V3 pMin, pMax;
    Box() {
        Float minNum = std::numeric_limits<Float>::lowest();
        Float maxNum = std::numeric_limits<Float>::max();
        pMin = V3(maxNum, maxNum, maxNum);
        pMax = V3(minNum, minNum, minNum);
    }
    // Bounds3(p1, p2) ctor: componentwise min / max   geometry.h:759-763
    Box(V3 p1, V3 p2) {
        pMin = V3(smin(p1.x, p2.x), smin(p1.y, p2.y), smin(p1.z, p2.z));
        pMax = V3(smax(p1.x, p2.x), smax(p1.y, p2.y), smax(p1.z, p2.z));
    }
    const V3 &operator[](int i) const { return i == 0 ? pMin : pMax; }
    V3 diagonal() const { return sub(pMax, pMin); }
    Float surfaceArea() const {
        V3 d = diagonal();
        return 2 * (d.x * d.y + d.x * d.z + d.y * d.z);
    }
    int maximumExtent() const {
        V3 d = diagonal();
        if (d.x > d.y && d.x > d.z) return 0;
        else if (d.y > d.z) return 1;
        else return 2;
    }
    // geometry.h:801-807 (true division here: o.x /= float)
    V3 offset(V3 p) const {
        V3 o = sub(p, pMin);
        if (pMax.x > pMin.x) o.x /= pMax.x - pMin.x;
        if (pMax.y > pMin.y) o.y /= pMax.y - pMin.y;
        if (pMax.z > pMin.z) o.z /= pMax.z - pMin.z;
        return o;
    }
};
// Union goes through the (p1,p2) ctor, geometry.h:1250-1266 (so Union(empty,empty) = everything)
static inline Box unionBB(const Box &b1, const Box &b2) {
    return Box(V3(smin(b1.pMin.x, b2.pMin.x), smin(b1.pMin.y, b2.pMin.y), smin(b1.pMin.z, b2.pMin.z)),
               V3(smax(b1.pMax.x, b2.pMax.x), smax(b1.pMax.y, b2.pMax.y), smax(b1.pMax.z, b2.pMax.z)));
}
static inline Box unionBP(const Box &b, V3 p) {
    return Box(V3(smin(b.pMin.x, p.x), smin(b.pMin.y, p.y), smin(b.pMin.z, p.z)),
               V3(smax(b.pMax.x, p.x), smax(b.pMax.y, p.y), smax(b.pMax.z, p.z)));
}

// gamma(n) pbrt.h:263-265 with MachineEpsilon = FLT_EPSILON*0.5 (pbrt.h:175-176)
static inline Float gammaN(int n) {
    const Float MachineEpsilon = std::numeric_limits<Float>::epsilon() * 0.5;
    return (n * MachineEpsilon) / (1 - n * MachineEpsilon);
}

struct PhotonBeam {  // photonbeambvh.h:48-73
    V3 start, end;
    Float radius;
    V3 powerStart, powerEnd;
    Box worldBound(int sqrtMode) const {
        V3 dir = sub(end, start);
        const V3 center = add(start, divv(dir, 2));
        const Float len = length(dir);
        dir = divv(dir, len);
        V3 size;
        if (sqrtMode == 0) {
            // libstdc++ reading: ::sqrt(double); product and sum in double, one rounding to float
            size.x = (Float)((double)(dir.x * len) + (double)(2 * radius) * ::sqrt((double)(1 - dir.x * dir.x)));
            size.y = (Float)((double)(dir.y * len) + (double)(2 * radius) * ::sqrt((double)(1 - dir.y * dir.y)));
            size.z = (Float)((double)(dir.z * len) + (double)(2 * radius) * ::sqrt((double)(1 - dir.z * dir.z)));
        } else {
            size.x = dir.x * len + 2 * radius * std::sqrt((Float)(1 - dir.x * dir.x));
            size.y = dir.y * len + 2 * radius * std::sqrt((Float)(1 - dir.y * dir.y));
            size.z = dir.z * len + 2 * radius * std::sqrt((Float)(1 - dir.z * dir.z));
        }
        return Box(sub(center, divv(size, 2)), add(center, divv(size, 2)));
    }
};

struct Ray {
    V3 o, d;
    Float tMax;
};

// geometry.h:1410-1436
static inline bool intersectP(const Box &bounds, const Ray &ray, V3 invDir, const int dirIsNeg[3]) {
    const Float pad = 1 + 2 * gammaN(3);
    Float tMin = (bounds[dirIsNeg[0]].x - ray.o.x) * invDir.x;
    Float tMax = (bounds[1 - dirIsNeg[0]].x - ray.o.x) * invDir.x;
    Float tyMin = (bounds[dirIsNeg[1]].y - ray.o.y) * invDir.y;
    Float tyMax = (bounds[1 - dirIsNeg[1]].y - ray.o.y) * invDir.y;
    tMax *= pad;
    tyMax *= pad;
    if (tMin > tyMax || tyMin > tMax) return false;
    if (tyMin > tMin) tMin = tyMin;
    if (tyMax < tMax) tMax = tyMax;
    Float tzMin = (bounds[dirIsNeg[2]].z - ray.o.z) * invDir.z;
    Float tzMax = (bounds[1 - dirIsNeg[2]].z - ray.o.z) * invDir.z;
    tzMax *= pad;
    if (tMin > tzMax || tzMin > tMax) return false;
    if (tzMin > tMin) tMin = tzMin;
    if (tzMax < tMax) tMax = tzMax;
    return (tMin < ray.tMax) && (tMax > 0);
}

// photonbeam.cpp:79-85
static inline Float determinant(V3 a, V3 b, V3 c) {
    return a.x * b.y * c.z + a.y * b.z * c.x + a.z * b.x * c.y -
           (a.z * b.y * c.x + a.y * b.x * c.z + a.x * b.z * c.y);
}

// photonbeam.cpp:87-186 (the dead `fabs` branches of the parallel case assign the same values)
static bool computeClosestPoints(V3 a0, V3 a1, V3 b0, V3 b1, V3 &aClosest, V3 &bClosest) {
    V3 A = sub(a1, a0);
    V3 B = sub(b1, b0);
    Float magA = length(A);
    Float magB = length(B);
    if (magA == 0.0f) {
        aClosest = a0;
        if (magB == 0.0f) {
            bClosest = b0;
            return true;
        }
        B = divv(B, magB);
        A = sub(a0, b0);
        Float d = dot(A, B);
        bClosest = add(b0, mul(B, Clamp(d, 0.0f, magB)));
        return true;
    } else if (magB == 0.0f) {
        bClosest = b0;
        A = divv(A, magA);
        B = sub(b0, a0);
        Float d = dot(A, B);
        aClosest = add(a0, mul(A, Clamp(d, 0.0f, magA)));
        return true;
    }
    A = divv(A, magA);
    B = divv(B, magB);
    const V3 cr = cross(A, B);
    const Float denom = lengthSq(cr);
    if (denom == Float(0.0f)) {
        Float d0 = dot(A, sub(b0, a0));
        Float d1 = dot(A, sub(b1, a0));
        if (d0 <= 0 && d1 <= 0) {
            aClosest = a0;
            bClosest = b1;
        } else if (d0 >= magA && d1 >= magA) {
            aClosest = a1;
            bClosest = b1;
        }
        return false;
    }
    const V3 t = sub(b0, a0);
    const Float detA = determinant(t, B, cr);
    const Float detB = determinant(t, A, cr);
    const Float t0 = detA / denom;
    const Float t1 = detB / denom;
    V3 pA = add(a0, mul(A, t0));
    V3 pB = add(b0, mul(B, t1));
    if (t0 < 0) pA = a0;
    else if (t0 > magA) pA = a1;
    if (t0 < 0 || t0 > magA) {
        Float d = Clamp(dot(B, sub(pA, b0)), 0.0f, magB);
        pB = add(b0, mul(B, d));
    }
    if (t1 < 0 || t1 > magB) {
        Float d = Clamp(dot(A, sub(pB, a0)), 0.0f, magA);
        pA = add(a0, mul(A, d));
    }
    aClosest = pA;
    bClosest = pB;
    return true;
}

// One beam's contribution to one camera segment, photonbeam.cpp:499-506.
// Returns true if it adds (and writes the RGB increment).
static inline bool beamContribution(const PhotonBeam &beam, V3 o, V3 p, Float currentBeamRadius,
                                    Float rgb[3]) {
    V3 rayClose, beamClose;
    if (!computeClosestPoints(o, p, beam.start, beam.end, rayClose, beamClose)) return false;
    const Float MaxDistance = currentBeamRadius + beam.radius;
    Float distance = length(sub(rayClose, beamClose));
    if (!(distance < MaxDistance)) return false;
    Float r = distance / MaxDistance;
    // `1e-5 * powerEnd` -> operator*(Float, Spectrum) with (Float)1e-5; then * sqrt(...)
    const Float k = (Float)1e-5;
    const Float w = (Float)::sqrt((double)(1.0f - r * r));  // == correctly rounded sqrtf
    rgb[0] = (beam.powerEnd.x * k) * w;
    rgb[1] = (beam.powerEnd.y * k) * w;
    rgb[2] = (beam.powerEnd.z * k) * w;
    return true;
}

// ---------------------------------------------------------------- SAH BVH (photonbeambvh.cpp)
struct BVHBeamInfo {  // :48-59
    size_t primitiveNumber;
    Box bounds;
    V3 centroid;
};
struct BuildNode {  // :61-85
    Box bounds;
    BuildNode *children[2];
    int splitAxis, firstPrimOffset, nPhotonBeams;
};
struct LinearNode {  // :97-106, 32 bytes
    Box bounds;
    union {
        int photonBeamsOffset;
        int secondChildOffset;
    };
    uint16_t nPhotonBeams;
    uint8_t axis;
    uint8_t pad[1];
};
static_assert(sizeof(LinearNode) == 32, "LinearPBBVHNode is 32 bytes in the reference");

struct BucketInfo {
    int count = 0;
    Box bounds;
};

class BeamBVH {
  public:
    BeamBVH(std::vector<std::shared_ptr<PhotonBeam>> &&beams, int sqrtMode)
        : maxPrimsInNode(1), photonBeams(std::move(beams)) {
        if (photonBeams.empty()) return;
        std::vector<BVHBeamInfo> info(photonBeams.size());
        for (size_t i = 0; i < photonBeams.size(); ++i) {
            Box b = photonBeams[i]->worldBound(sqrtMode);
            info[i].primitiveNumber = i;
            info[i].bounds = b;
            // .5f * pMin + .5f * pMax   (:51-54)
            info[i].centroid = add(mul(b.pMin, .5f), mul(b.pMax, .5f));
        }
        std::vector<std::unique_ptr<BuildNode>> arena;
        int totalNodes = 0;
        std::vector<std::shared_ptr<PhotonBeam>> ordered;
        ordered.reserve(photonBeams.size());
        BuildNode *root = recursiveBuild(arena, info, 0, (int)photonBeams.size(), &totalNodes, ordered);
        photonBeams.swap(ordered);
        nodes.resize(totalNodes);
        int offset = 0;
        flatten(root, &offset);
    }

    // :685-723; V = nodes whose bounds were tested
    std::vector<std::shared_ptr<PhotonBeam>> intersect(const Ray &ray, int64_t *visited) const {
        std::vector<std::shared_ptr<PhotonBeam>> beams;
        if (nodes.empty()) return beams;
        V3 invDir(1 / ray.d.x, 1 / ray.d.y, 1 / ray.d.z);
        int dirIsNeg[3] = {invDir.x < 0, invDir.y < 0, invDir.z < 0};
        int toVisitOffset = 0, currentNodeIndex = 0;
        int nodesToVisit[64];
        int64_t v = 0;
        while (true) {
            const LinearNode *node = &nodes[currentNodeIndex];
            ++v;
            if (intersectP(node->bounds, ray, invDir, dirIsNeg)) {
                if (node->nPhotonBeams > 0) {
                    for (int i = 0; i < node->nPhotonBeams; ++i)
                        beams.push_back(photonBeams[node->photonBeamsOffset + i]);
                    if (toVisitOffset == 0) break;
                    currentNodeIndex = nodesToVisit[--toVisitOffset];
                } else {
                    if (dirIsNeg[node->axis]) {
                        nodesToVisit[toVisitOffset++] = currentNodeIndex + 1;
                        currentNodeIndex = node->secondChildOffset;
                    } else {
                        nodesToVisit[toVisitOffset++] = node->secondChildOffset;
                        currentNodeIndex = currentNodeIndex + 1;
                    }
                }
            } else {
                if (toVisitOffset == 0) break;
                currentNodeIndex = nodesToVisit[--toVisitOffset];
            }
        }
        if (visited) *visited = v;
        return beams;
    }
    // The same depth-first walk as intersect(), handing each leaf beam to f in the order intersect()
    // would return it, without building the per-query vector<shared_ptr> (image-parity mode, below).
    template <class F>
    void forEachCandidate(const Ray &ray, F &&f, int64_t *visited) const {
        if (nodes.empty()) return;
        V3 invDir(1 / ray.d.x, 1 / ray.d.y, 1 / ray.d.z);
        int dirIsNeg[3] = {invDir.x < 0, invDir.y < 0, invDir.z < 0};
        int toVisitOffset = 0, currentNodeIndex = 0;
        int nodesToVisit[64];
        int64_t v = 0;
        while (true) {
            const LinearNode *node = &nodes[currentNodeIndex];
            ++v;
            if (intersectP(node->bounds, ray, invDir, dirIsNeg)) {
                if (node->nPhotonBeams > 0) {
                    for (int i = 0; i < node->nPhotonBeams; ++i) f(*photonBeams[node->photonBeamsOffset + i]);
                    if (toVisitOffset == 0) break;
                    currentNodeIndex = nodesToVisit[--toVisitOffset];
                } else {
                    if (dirIsNeg[node->axis]) {
                        nodesToVisit[toVisitOffset++] = currentNodeIndex + 1;
                        currentNodeIndex = node->secondChildOffset;
                    } else {
                        nodesToVisit[toVisitOffset++] = node->secondChildOffset;
                        currentNodeIndex = currentNodeIndex + 1;
                    }
                }
            } else {
                if (toVisitOffset == 0) break;
                currentNodeIndex = nodesToVisit[--toVisitOffset];
            }
        }
        if (visited) *visited = v;
    }
    size_t nodeCount() const { return nodes.size(); }
    size_t beamCount() const { return photonBeams.size(); }
    int maxLeafSize() const {
        int m = 0;
        for (const LinearNode &n : nodes) m = std::max(m, (int)n.nPhotonBeams);
        return m;
    }

  private:
    BuildNode *newNode(std::vector<std::unique_ptr<BuildNode>> &arena) {
        arena.emplace_back(new BuildNode());
        return arena.back().get();
    }
    void initLeaf(BuildNode *n, int first, int cnt, const Box &b) {
        n->firstPrimOffset = first;
        n->nPhotonBeams = cnt;
        n->bounds = b;
        n->children[0] = n->children[1] = nullptr;
    }
    void emitLeaf(BuildNode *node, std::vector<BVHBeamInfo> &info, int start, int end, const Box &bounds,
                  std::vector<std::shared_ptr<PhotonBeam>> &ordered) {
        int first = (int)ordered.size();
        for (int i = start; i < end; ++i) ordered.push_back(photonBeams[info[i].primitiveNumber]);
        initLeaf(node, first, end - start, bounds);
    }
    // :259-425 (SplitMethod::SAH branch)
    BuildNode *recursiveBuild(std::vector<std::unique_ptr<BuildNode>> &arena, std::vector<BVHBeamInfo> &info,
                              int start, int end, int *totalNodes,
                              std::vector<std::shared_ptr<PhotonBeam>> &ordered) {
        BuildNode *node = newNode(arena);
        (*totalNodes)++;
        Box bounds;
        for (int i = start; i < end; ++i) bounds = unionBB(bounds, info[i].bounds);
        int n = end - start;
        if (n == 1) {
            emitLeaf(node, info, start, end, bounds, ordered);
            return node;
        }
        Box centroidBounds;
        for (int i = start; i < end; ++i) centroidBounds = unionBP(centroidBounds, info[i].centroid);
        int dim = centroidBounds.maximumExtent();
        int mid = (start + end) / 2;
        if (centroidBounds.pMax[dim] == centroidBounds.pMin[dim]) {
            emitLeaf(node, info, start, end, bounds, ordered);
            return node;
        }
        if (n <= 2) {
            mid = (start + end) / 2;
            std::nth_element(&info[start], &info[mid], &info[end - 1] + 1,
                             [dim](const BVHBeamInfo &a, const BVHBeamInfo &b) {
                                 return a.centroid[dim] < b.centroid[dim];
                             });
        } else {
            const int nBuckets = 12;
            BucketInfo buckets[nBuckets];
            for (int i = start; i < end; ++i) {
                int b = (int)(nBuckets * centroidBounds.offset(info[i].centroid)[dim]);
                if (b == nBuckets) b = nBuckets - 1;
                buckets[b].count++;
                buckets[b].bounds = unionBB(buckets[b].bounds, info[i].bounds);
            }
            Float cost[nBuckets - 1];
            for (int i = 0; i < nBuckets - 1; ++i) {
                Box b0, b1;
                int count0 = 0, count1 = 0;
                for (int j = 0; j <= i; ++j) {
                    b0 = unionBB(b0, buckets[j].bounds);
                    count0 += buckets[j].count;
                }
                for (int j = i + 1; j < nBuckets; ++j) {
                    b1 = unionBB(b1, buckets[j].bounds);
                    count1 += buckets[j].count;
                }
                cost[i] = 1 + (count0 * b0.surfaceArea() + count1 * b1.surfaceArea()) / bounds.surfaceArea();
            }
            Float minCost = cost[0];
            int minCostSplitBucket = 0;
            for (int i = 1; i < nBuckets - 1; ++i) {
                if (cost[i] < minCost) {
                    minCost = cost[i];
                    minCostSplitBucket = i;
                }
            }
            Float leafCost = n;
            if (n > maxPrimsInNode || minCost < leafCost) {
                BVHBeamInfo *pmid = std::partition(&info[start], &info[end - 1] + 1, [=](const BVHBeamInfo &pi) {
                    int b = (int)(nBuckets * centroidBounds.offset(pi.centroid)[dim]);
                    if (b == nBuckets) b = nBuckets - 1;
                    return b <= minCostSplitBucket;
                });
                mid = (int)(pmid - &info[0]);
            } else {
                emitLeaf(node, info, start, end, bounds, ordered);
                return node;
            }
        }
        BuildNode *c0 = recursiveBuild(arena, info, start, mid, totalNodes, ordered);
        BuildNode *c1 = recursiveBuild(arena, info, mid, end, totalNodes, ordered);
        node->children[0] = c0;
        node->children[1] = c1;
        node->bounds = unionBB(c0->bounds, c1->bounds);
        node->splitAxis = dim;
        node->nPhotonBeams = 0;
        return node;
    }
    int flatten(BuildNode *node, int *offset) {  // :663-681
        LinearNode *ln = &nodes[*offset];
        ln->bounds = node->bounds;
        int myOffset = (*offset)++;
        if (node->nPhotonBeams > 0) {
            ln->photonBeamsOffset = node->firstPrimOffset;
            ln->nPhotonBeams = (uint16_t)node->nPhotonBeams;
        } else {
            ln->axis = (uint8_t)node->splitAxis;
            ln->nPhotonBeams = 0;
            flatten(node->children[0], offset);
            ln = &nodes[myOffset];
            ln->secondChildOffset = flatten(node->children[1], offset);
        }
        return myOffset;
    }

    const int maxPrimsInNode;
    std::vector<std::shared_ptr<PhotonBeam>> photonBeams;
    std::vector<LinearNode> nodes;
};

static inline V3 ld3(const float *p, int64_t i) { return V3(p[3 * i], p[3 * i + 1], p[3 * i + 2]); }

struct Handle {
    BeamBVH *bvh = nullptr;
    std::vector<std::shared_ptr<PhotonBeam>> beamsInInputOrder;
    int sqrtMode = 0;
};

// Gather for one segment through the reference tree, photonbeam.cpp:494-508.
static void gatherSegment(const BeamBVH &bvh, V3 o, V3 p, V3 d, Float tMax, Float R, Float *acc /*+=*/,
                          int64_t *cand, int64_t *vis, int64_t *contrib) {
    Ray ray{o, d, tMax};
    int64_t v = 0;
    std::vector<std::shared_ptr<PhotonBeam>> beams = bvh.intersect(ray, &v);
    int64_t nc = 0;
    for (std::shared_ptr<PhotonBeam> const &beam : beams) {
        Float rgb[3];
        if (beamContribution(*beam, o, p, R, rgb)) {
            acc[0] += rgb[0];
            acc[1] += rgb[1];
            acc[2] += rgb[2];
            ++nc;
        }
    }
    if (cand) *cand = (int64_t)beams.size();
    if (vis) *vis = v;
    if (contrib) *contrib = nc;
}

// Image-parity mode (tests only: whole films at BASELINE sizes, where the reference form takes tens
// of minutes).  The candidates come in the reference's DFS order and every candidate that can
// contribute goes through beamContribution exactly as above, so the sums and counts are ora_gather's
// bit for bit.  A candidate is skipped without ComputeClosestPoints only when the double-precision
// distance D between the segment's LINE and the beam's LINE exceeds MaxDistance by 1e-4 (1 + the
// coordinate scale): the reference's aClosest lies on segment A and its bClosest on beam B's line
// (also in the t1 quirk of photonbeam.cpp:178-181), each to within a few float ulps of the
// coordinates and of |t1| <= |t| / |n| (<= 100 x the scale for |n| >= 0.01, the only pairs skipped),
// so its float distance is >= D - 1e-5 (1 + scale) > MaxDistance: such a pair never contributes.
static void gatherSegmentSkip(const BeamBVH &bvh, V3 o, V3 p, V3 d, Float tMax, Float R, Float *acc,
                              int64_t *cand, int64_t *vis, int64_t *contrib, int64_t *skipped) {
    Ray ray{o, d, tMax};
    int64_t v = 0, nc = 0, nk = 0, ns = 0;
    const double ax = (double)p.x - o.x, ay = (double)p.y - o.y, az = (double)p.z - o.z;
    const double al = std::sqrt(ax * ax + ay * ay + az * az);
    const double osc = std::max(std::max(std::fabs((double)o.x), std::fabs((double)o.y)), std::fabs((double)o.z)) + al;
    bvh.forEachCandidate(ray, [&](const PhotonBeam &beam) {
        ++nc;
        const double bx = (double)beam.end.x - beam.start.x, by = (double)beam.end.y - beam.start.y,
                     bz = (double)beam.end.z - beam.start.z;
        const double bl = std::sqrt(bx * bx + by * by + bz * bz);
        if (al > 0 && bl > 0) {
            const double ux = ax / al, uy = ay / al, uz = az / al, vx = bx / bl, vy = by / bl, vz = bz / bl;
            const double nx = uy * vz - uz * vy, ny = uz * vx - ux * vz, nz = ux * vy - uy * vx;
            const double nl = std::sqrt(nx * nx + ny * ny + nz * nz);
            if (nl >= 0.01) {
                const double tx = (double)beam.start.x - o.x, ty = (double)beam.start.y - o.y,
                             tz = (double)beam.start.z - o.z;
                const double D = std::fabs(tx * nx + ty * ny + tz * nz) / nl;
                const double bsc = std::max(std::max(std::fabs((double)beam.start.x), std::fabs((double)beam.start.y)),
                                            std::fabs((double)beam.start.z)) + bl;
                if (D > (double)(R + beam.radius) + 1e-4 * (1.0 + osc + bsc)) {
                    ++ns;
                    return;
                }
            }
        }
        Float rgb[3];
        if (beamContribution(beam, o, p, R, rgb)) {
            acc[0] += rgb[0];
            acc[1] += rgb[1];
            acc[2] += rgb[2];
            ++nk;
        }
    }, &v);
    if (cand) *cand = nc;
    if (vis) *vis = v;
    if (contrib) *contrib = nk;
    if (skipped) *skipped = ns;
}

}  // namespace ora

using namespace ora;

extern "C" {

int ora_version(void) { return 1; }

// 1 + 2*gamma(3) as the reference computes it in Float.
float ora_slab_pad(void) { return 1 + 2 * gammaN(3); }

void ora_beam_bounds(int64_t n, const float *start, const float *end, const float *radius, int sqrtMode,
                     float *box /* 6n: min xyz, max xyz */) {
    for (int64_t i = 0; i < n; ++i) {
        PhotonBeam b;
        b.start = ld3(start, i);
        b.end = ld3(end, i);
        b.radius = radius[i];
        Box bb = b.worldBound(sqrtMode);
        box[6 * i + 0] = bb.pMin.x;
        box[6 * i + 1] = bb.pMin.y;
        box[6 * i + 2] = bb.pMin.z;
        box[6 * i + 3] = bb.pMax.x;
        box[6 * i + 4] = bb.pMax.y;
        box[6 * i + 5] = bb.pMax.z;
    }
}

int ora_closest_points(const float *a0, const float *a1, const float *b0, const float *b1, float *aC, float *bC) {
    V3 pa, pb;
    bool ok = computeClosestPoints(V3(a0[0], a0[1], a0[2]), V3(a1[0], a1[1], a1[2]), V3(b0[0], b0[1], b0[2]),
                                   V3(b1[0], b1[1], b1[2]), pa, pb);
    aC[0] = pa.x; aC[1] = pa.y; aC[2] = pa.z;
    bC[0] = pb.x; bC[1] = pb.y; bC[2] = pb.z;
    return ok ? 1 : 0;
}

int ora_intersect_box(const float *box, const float *o, const float *d, float tMax) {
    Box b;
    b.pMin = V3(box[0], box[1], box[2]);
    b.pMax = V3(box[3], box[4], box[5]);
    Ray ray{V3(o[0], o[1], o[2]), V3(d[0], d[1], d[2]), tMax};
    V3 invDir(1 / ray.d.x, 1 / ray.d.y, 1 / ray.d.z);
    int neg[3] = {invDir.x < 0, invDir.y < 0, invDir.z < 0};
    return intersectP(b, ray, invDir, neg) ? 1 : 0;
}

// Radius schedule, photonbeam.cpp:354-356 and :562.
float ora_radius_at(float initialRadius, float alpha, int iteration) {
    Float r = initialRadius;
    for (int i = 0; i < iteration; ++i) r = r * (Float(i + alpha) / Float(i + 1));
    return r;
}

void *ora_bvh_build(int64_t n, const float *start, const float *end, const float *radius, const float *powerEnd,
                    int sqrtMode) {
    Handle *h = new Handle();
    h->sqrtMode = sqrtMode;
    std::vector<std::shared_ptr<PhotonBeam>> beams;
    beams.reserve((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        auto b = std::make_shared<PhotonBeam>();
        b->start = ld3(start, i);
        b->end = ld3(end, i);
        b->radius = radius[i];
        b->powerStart = V3(0, 0, 0);  // photonbeam.cpp:266,292: betaStart default-constructed = 0
        b->powerEnd = ld3(powerEnd, i);
        beams.push_back(b);
    }
    h->beamsInInputOrder = beams;
    h->bvh = new BeamBVH(std::move(beams), sqrtMode);
    return h;
}

int64_t ora_bvh_node_count(void *hp) { return (int64_t)((Handle *)hp)->bvh->nodeCount(); }
int ora_bvh_max_leaf(void *hp) { return ((Handle *)hp)->bvh->maxLeafSize(); }

void ora_bvh_free(void *hp) {
    Handle *h = (Handle *)hp;
    if (!h) return;
    delete h->bvh;
    delete h;
}

// Gather through the reference tree.  Per segment outputs (any may be null): seg_rgb[3],
// seg_cand (C: beams returned by Intersect), seg_visit (V: nodes tested), seg_contrib.
// pix_rgb (if non-null) is accumulated exactly like PhotonBeamPixel::Ld in segment order
// (nthreads must be 1 for that).  nthreads>1 partitions segments into chunks of `chunk`
// (a 16x16 tile = 256) pulled dynamically, like ParallelFor2D over tiles.
void ora_gather(void *hp, int64_t nseg, const float *o, const float *p, const float *d, const float *tmax,
                const int32_t *pixel, float R, float *seg_rgb, float *pix_rgb, int64_t *seg_cand,
                int64_t *seg_visit, int64_t *seg_contrib, int nthreads, int64_t chunk) {
    Handle *h = (Handle *)hp;
    const BeamBVH &bvh = *h->bvh;
    if (nthreads <= 1 || pix_rgb) {
        for (int64_t s = 0; s < nseg; ++s) {
            Float acc[3] = {0, 0, 0};
            Float *dst = acc;
            if (pix_rgb && pixel) dst = pix_rgb + 3 * (int64_t)pixel[s];
            Float before[3] = {dst[0], dst[1], dst[2]};
            int64_t c, v, k;
            gatherSegment(bvh, ld3(o, s), ld3(p, s), ld3(d, s), tmax[s], R, dst, &c, &v, &k);
            if (seg_rgb) {
                if (dst == acc) {
                    seg_rgb[3 * s] = acc[0]; seg_rgb[3 * s + 1] = acc[1]; seg_rgb[3 * s + 2] = acc[2];
                } else {
                    seg_rgb[3 * s] = dst[0] - before[0];
                    seg_rgb[3 * s + 1] = dst[1] - before[1];
                    seg_rgb[3 * s + 2] = dst[2] - before[2];
                }
            }
            if (seg_cand) seg_cand[s] = c;
            if (seg_visit) seg_visit[s] = v;
            if (seg_contrib) seg_contrib[s] = k;
        }
        return;
    }
    if (chunk <= 0) chunk = 256;
    std::atomic<int64_t> next(0);
    auto worker = [&]() {
        while (true) {
            int64_t s0 = next.fetch_add(chunk);
            if (s0 >= nseg) break;
            int64_t s1 = std::min(nseg, s0 + chunk);
            for (int64_t s = s0; s < s1; ++s) {
                Float acc[3] = {0, 0, 0};
                int64_t c, v, k;
                gatherSegment(bvh, ld3(o, s), ld3(p, s), ld3(d, s), tmax[s], R, acc, &c, &v, &k);
                if (seg_rgb) {
                    seg_rgb[3 * s] = acc[0]; seg_rgb[3 * s + 1] = acc[1]; seg_rgb[3 * s + 2] = acc[2];
                }
                if (seg_cand) seg_cand[s] = c;
                if (seg_visit) seg_visit[s] = v;
                if (seg_contrib) seg_contrib[s] = k;
            }
        }
    };
    std::vector<std::thread> pool;
    for (int t = 0; t < nthreads; ++t) pool.emplace_back(worker);
    for (auto &t : pool) t.join();
}

// The image-parity gather (gatherSegmentSkip): ora_gather's per-segment sums, candidate and
// contribution counts bit for bit, on nthreads threads; seg_skip (optional) counts the candidates
// skipped by the line-distance proof.  Films are composed by the caller in segment order.
void ora_gather_skip(void *hp, int64_t nseg, const float *o, const float *p, const float *d, const float *tmax,
                     float R, float *seg_rgb, int64_t *seg_cand, int64_t *seg_contrib, int64_t *seg_skip,
                     int nthreads) {
    Handle *h = (Handle *)hp;
    const BeamBVH &bvh = *h->bvh;
    std::atomic<int64_t> next(0);
    const int64_t chunk = 64;
    auto worker = [&]() {
        while (true) {
            const int64_t s0 = next.fetch_add(chunk);
            if (s0 >= nseg) break;
            const int64_t s1 = std::min(nseg, s0 + chunk);
            for (int64_t s = s0; s < s1; ++s) {
                Float acc[3] = {0, 0, 0};
                int64_t c, v, k, sk;
                gatherSegmentSkip(bvh, ld3(o, s), ld3(p, s), ld3(d, s), tmax[s], R, acc, &c, &v, &k, &sk);
                if (seg_rgb) {
                    seg_rgb[3 * s] = acc[0]; seg_rgb[3 * s + 1] = acc[1]; seg_rgb[3 * s + 2] = acc[2];
                }
                if (seg_cand) seg_cand[s] = c;
                if (seg_contrib) seg_contrib[s] = k;
                if (seg_skip) seg_skip[s] = sk;
            }
        }
    };
    std::vector<std::thread> pool;
    for (int t = 0; t < std::max(1, nthreads); ++t) pool.emplace_back(worker);
    for (auto &t : pool) t.join();
}

// BVH-free restatement of the same candidate set: a beam is a candidate iff the box of its
// equal-centroid group (the reference's SAH leaf, photonbeambvh.cpp:289-297) passes
// IntersectP.  Beams are visited in input order.  Used to cross-check the tree and to pin
// the GPU's (BVH-independent) candidate set.
void ora_gather_bruteforce(int64_t nb, const float *start, const float *end, const float *radius,
                           const float *powerEnd, int sqrtMode, int64_t nseg, const float *o, const float *p,
                           const float *d, const float *tmax, float R, float *seg_rgb, int64_t *seg_cand,
                           int64_t *seg_contrib, int nthreads, double *seg_rgb_exact) {
    std::vector<PhotonBeam> beams((size_t)nb);
    std::vector<Box> boxes((size_t)nb);
    std::vector<V3> cent((size_t)nb);
    for (int64_t i = 0; i < nb; ++i) {
        beams[i].start = ld3(start, i);
        beams[i].end = ld3(end, i);
        beams[i].radius = radius[i];
        beams[i].powerEnd = ld3(powerEnd, i);
        boxes[i] = beams[i].worldBound(sqrtMode);
        cent[i] = add(mul(boxes[i].pMin, .5f), mul(boxes[i].pMax, .5f));
    }
    // group boxes: union over beams with identical (==) centroid
    std::vector<int64_t> order((size_t)nb);
    for (int64_t i = 0; i < nb; ++i) order[i] = i;
    auto key_less = [&](int64_t a, int64_t b) {
        if (cent[a].x != cent[b].x) return cent[a].x < cent[b].x;
        if (cent[a].y != cent[b].y) return cent[a].y < cent[b].y;
        return cent[a].z < cent[b].z;
    };
    auto nan3 = [&](int64_t i) { return std::isnan(cent[i].x) || std::isnan(cent[i].y) || std::isnan(cent[i].z); };
    std::vector<int64_t> finite;
    for (int64_t i = 0; i < nb; ++i)
        if (!nan3(i)) finite.push_back(i);
    std::sort(finite.begin(), finite.end(), key_less);
    std::vector<Box> gbox = boxes;
    for (size_t a = 0; a < finite.size();) {
        size_t b = a + 1;
        while (b < finite.size() && cent[finite[b]].x == cent[finite[a]].x &&
               cent[finite[b]].y == cent[finite[a]].y && cent[finite[b]].z == cent[finite[a]].z)
            ++b;
        if (b - a > 1) {
            Box u;
            for (size_t k = a; k < b; ++k) u = unionBB(u, boxes[finite[k]]);
            for (size_t k = a; k < b; ++k) gbox[finite[k]] = u;
        }
        a = b;
    }
    // segments are independent: nthreads workers take segments in turn (each segment's sum is
    // still in input order, so the result does not depend on nthreads)
    std::atomic<int64_t> next(0);
    auto worker = [&]() {
        for (int64_t s; (s = next.fetch_add(1)) < nseg;) {
            Ray ray{ld3(o, s), ld3(d, s), tmax[s]};
            V3 invDir(1 / ray.d.x, 1 / ray.d.y, 1 / ray.d.z);
            int neg[3] = {invDir.x < 0, invDir.y < 0, invDir.z < 0};
            Float acc[3] = {0, 0, 0};
            double dacc[3] = {0, 0, 0};  // the same float terms summed in double (test reference)
            int64_t c = 0, k = 0;
            V3 pp = ld3(p, s);
            for (int64_t i = 0; i < nb; ++i) {
                if (!intersectP(gbox[i], ray, invDir, neg)) continue;
                ++c;
                Float rgb[3];
                if (beamContribution(beams[i], ray.o, pp, R, rgb)) {
                    acc[0] += rgb[0]; acc[1] += rgb[1]; acc[2] += rgb[2];
                    dacc[0] += rgb[0]; dacc[1] += rgb[1]; dacc[2] += rgb[2];
                    ++k;
                }
            }
            if (seg_rgb) { seg_rgb[3 * s] = acc[0]; seg_rgb[3 * s + 1] = acc[1]; seg_rgb[3 * s + 2] = acc[2]; }
            if (seg_rgb_exact)
                for (int q = 0; q < 3; ++q) seg_rgb_exact[3 * s + q] = dacc[q];
            if (seg_cand) seg_cand[s] = c;
            if (seg_contrib) seg_contrib[s] = k;
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < nthreads; ++t) pool.emplace_back(worker);
    worker();
    for (auto &t : pool) t.join();
}

}  // extern "C"
