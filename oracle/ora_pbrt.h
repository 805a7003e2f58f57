// ora_pbrt.h — pbrt building blocks restated for the oracle's photon and camera passes
// (TEST INFRASTRUCTURE; see bre_oracle_photon.cpp for the file:line list and interpretation notes).
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <memory>
#include <vector>

#include "../include/bre_fmath.h"
#include "../include/bre_scene.h"

namespace orp {

typedef float Float;
static const Float Pi = 3.14159265358979323846f;
static const Float InvPi = 0.31830988618379067154f;
static const Float Inv4Pi = 0.07957747154594766788f;
static const Float PiOver2 = 1.57079632679489661923f;
static const Float PiOver4 = 0.78539816339744830961f;
static const Float OneMinusEpsilon = 0x1.fffffep-1f;
static const Float MachineEpsilon = 0x1p-24f;
static const Float Infinity = __builtin_huge_valf();
static const Float MaxFloat = 3.402823466e+38f;

static inline Float gamma(int n) { return (n * MachineEpsilon) / (1 - n * MachineEpsilon); }

// Transcendentals.  By default the oracle uses the same restatements as the GPU
// (include/bre_fmath.h) so photon and camera paths agree bit for bit; with ora_set_libm(1) it calls
// the host libm (std::exp / std::log / std::sin / std::cos) as the reference does
// (spectrum.h:222-224, homogeneous.cpp:47, grid.cpp:76,104, sampling.cpp:127).  Since round 6
// bre_fmath.h returns libm's bits for every float input (tests/test_fmath_libm.py), so the switch
// changes nothing (tests/test_faithful.py holds that).
extern int g_ora_libm;
static inline Float ora_exp(Float x) { return g_ora_libm ? std::exp(x) : bre_expf(x); }
static inline Float ora_log(Float x) { return g_ora_libm ? std::log(x) : bre_logf(x); }
static inline void ora_sincos(Float x, Float *s, Float *c) {
    if (g_ora_libm) {
        *s = std::sin(x);
        *c = std::cos(x);
    } else {
        bre_sincosf(x, s, c);
    }
}

// ---- RNG (rng.h:60-144) ----
struct RNG {
    uint64_t state, inc;
    RNG() : state(0x853c49e6748fea9bULL), inc(0xda3e39cb94b95bdbULL) {}  // PCG32_DEFAULT_STATE/STREAM
    explicit RNG(uint64_t seq) { SetSequence(seq); }
    uint32_t UniformUInt32(uint32_t b) {
        uint32_t threshold = (~b + 1u) % b;
        while (true) {
            uint32_t r = UniformUInt32();
            if (r >= threshold) return r % b;
        }
    }
    void SetSequence(uint64_t initseq) {
        state = 0u;
        inc = (initseq << 1u) | 1u;
        UniformUInt32();
        state += 0x853c49e6748fea9bULL;
        UniformUInt32();
    }
    uint32_t UniformUInt32() {
        uint64_t oldstate = state;
        state = oldstate * 0x5851f42d4c957f2dULL + inc;
        uint32_t xorshifted = (uint32_t)(((oldstate >> 18u) ^ oldstate) >> 27u);
        uint32_t rot = (uint32_t)(oldstate >> 59u);
        return (xorshifted >> rot) | (xorshifted << ((~rot + 1u) & 31));
    }
    Float UniformFloat() {
        return std::min(OneMinusEpsilon, Float(UniformUInt32() * 0x1p-32f));
    }
};

// AwesomeHaltonSampler past its 1000 Halton dimensions (photonbeam.cpp:226-256)
struct Sampler {
    RNG rng;
    explicit Sampler(uint64_t seq) : rng(seq) {}
    Float Get1D() { return rng.UniformFloat(); }
    void Get2D(Float *x, Float *y) {
        Float first = Get1D();
        Float second = Get1D();
        *x = second;  // g++ evaluates Point2f(Get1D(), Get1D()) right to left
        *y = first;
    }
};

// ---- geometry (geometry.h) ----
struct V3 {
    Float x, y, z;
    V3() : x(0), y(0), z(0) {}
    V3(Float a, Float b, Float c) : x(a), y(b), z(c) {}
    explicit V3(const float *p) : x(p[0]), y(p[1]), z(p[2]) {}
    Float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
    Float &operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
    V3 operator+(const V3 &b) const { return V3(x + b.x, y + b.y, z + b.z); }
    V3 operator-(const V3 &b) const { return V3(x - b.x, y - b.y, z - b.z); }
    V3 operator-() const { return V3(-x, -y, -z); }
    V3 operator*(Float s) const { return V3(s * x, s * y, s * z); }
    V3 operator/(Float f) const {
        Float inv = (Float)1 / f;
        return V3(x * inv, y * inv, z * inv);
    }
    Float LengthSquared() const { return x * x + y * y + z * z; }
    Float Length() const { return std::sqrt(LengthSquared()); }
};
static inline V3 operator*(Float s, const V3 &v) { return v * s; }
static inline Float Dot(const V3 &a, const V3 &b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline Float AbsDot(const V3 &a, const V3 &b) { return std::fabs(Dot(a, b)); }
static inline V3 Abs(const V3 &a) { return V3(std::fabs(a.x), std::fabs(a.y), std::fabs(a.z)); }
static inline V3 Normalize(const V3 &v) { return v / v.Length(); }
// Cross in double (geometry.h:957-963)
static inline V3 Cross(const V3 &v1, const V3 &v2) {
    double v1x = v1.x, v1y = v1.y, v1z = v1.z;
    double v2x = v2.x, v2y = v2.y, v2z = v2.z;
    return V3((Float)((v1y * v2z) - (v1z * v2y)), (Float)((v1z * v2x) - (v1x * v2z)),
              (Float)((v1x * v2y) - (v1y * v2x)));
}
static inline void CoordinateSystem(const V3 &v1, V3 *v2, V3 *v3) {
    if (std::fabs(v1.x) > std::fabs(v1.y))
        *v2 = V3(-v1.z, 0, v1.x) / std::sqrt(v1.x * v1.x + v1.z * v1.z);
    else
        *v2 = V3(0, v1.z, -v1.y) / std::sqrt(v1.y * v1.y + v1.z * v1.z);
    *v3 = Cross(v1, *v2);
}
static inline Float NextFloatUp(Float v) {
    if (std::isinf(v) && v > 0.) return v;
    if (v == -0.f) v = 0.f;
    uint32_t ui = bre_f2u(v);
    if (v >= 0) ++ui;
    else --ui;
    return bre_u2f(ui);
}
static inline Float NextFloatDown(Float v) {
    if (std::isinf(v) && v < 0.) return v;
    if (v == 0.f) v = -0.f;
    uint32_t ui = bre_f2u(v);
    if (v > 0) --ui;
    else ++ui;
    return bre_u2f(ui);
}
static inline V3 OffsetRayOrigin(const V3 &p, const V3 &pError, const V3 &n, const V3 &w) {
    Float d = Dot(Abs(n), pError);
    V3 offset = d * n;
    if (Dot(w, n) < 0) offset = -offset;
    V3 po = p + offset;
    for (int i = 0; i < 3; ++i) {
        if (offset[i] > 0) po[i] = NextFloatUp(po[i]);
        else if (offset[i] < 0) po[i] = NextFloatDown(po[i]);
    }
    return po;
}

// ---- RGBSpectrum (spectrum.h) ----
struct Spectrum {
    Float c[3];
    Spectrum(Float v = 0.f) { c[0] = c[1] = c[2] = v; }
    Spectrum(Float a, Float b, Float d) {
        c[0] = a;
        c[1] = b;
        c[2] = d;
    }
    explicit Spectrum(const float *p) : Spectrum(p[0], p[1], p[2]) {}
    Spectrum operator*(const Spectrum &o) const { return Spectrum(c[0] * o.c[0], c[1] * o.c[1], c[2] * o.c[2]); }
    Spectrum operator*(Float a) const { return Spectrum(c[0] * a, c[1] * a, c[2] * a); }
    Spectrum operator/(Float a) const { return Spectrum(c[0] / a, c[1] / a, c[2] / a); }
    Spectrum operator+(const Spectrum &o) const { return Spectrum(c[0] + o.c[0], c[1] + o.c[1], c[2] + o.c[2]); }
    Spectrum operator-() const { return Spectrum(-c[0], -c[1], -c[2]); }
    bool IsBlack() const { return c[0] == 0 && c[1] == 0 && c[2] == 0; }
    Float y() const { return 0.212671f * c[0] + 0.715160f * c[1] + 0.072169f * c[2]; }
};
static inline Spectrum operator*(Float a, const Spectrum &s) { return s * a; }
static inline Spectrum Exp(const Spectrum &s) {
    return Spectrum(ora_exp(s.c[0]), ora_exp(s.c[1]), ora_exp(s.c[2]));
}

// ---- sampling (sampling.cpp:113-133, sampling.h:159-165) ----
static inline void ConcentricSampleDisk(Float ux, Float uy, Float *dx, Float *dy) {
    Float ox = 2.f * ux - 1, oy = 2.f * uy - 1;
    if (ox == 0 && oy == 0) {
        *dx = 0;
        *dy = 0;
        return;
    }
    Float theta, r;
    if (std::fabs(ox) > std::fabs(oy)) {
        r = ox;
        theta = PiOver4 * (oy / ox);
    } else {
        r = oy;
        theta = PiOver2 - PiOver4 * (ox / oy);
    }
    Float s, c;
    ora_sincos(theta, &s, &c);
    *dx = c * r;
    *dy = s * r;
}
static inline V3 CosineSampleHemisphere(Float ux, Float uy) {
    Float dx, dy;
    ConcentricSampleDisk(ux, uy, &dx, &dy);
    Float z = std::sqrt(std::max((Float)0, 1 - dx * dx - dy * dy));
    return V3(dx, dy, z);
}

// ---- Henyey-Greenstein (medium.cpp:194-218, medium.h:69-72) ----
static inline Float PhaseHG(Float cosTheta, Float g) {
    Float denom = 1 + g * g + 2 * g * cosTheta;
    return Inv4Pi * (1 - g * g) / (denom * std::sqrt(denom));
}
static inline Float HG_Sample_p(Float g, const V3 &wo, V3 *wi, Float u0, Float u1) {
    Float cosTheta;
    if (std::abs(g) < 1e-3)
        cosTheta = 1 - 2 * u0;
    else {
        Float sqrTerm = (1 - g * g) / (1 - g + 2 * g * u0);
        cosTheta = (1 + g * g - sqrTerm * sqrTerm) / (2 * g);
    }
    Float sinTheta = std::sqrt(std::max((Float)0, 1 - cosTheta * cosTheta));
    Float phi = 2 * Pi * u1;
    V3 v1, v2;
    CoordinateSystem(wo, &v1, &v2);
    Float sp, cp;
    ora_sincos(phi, &sp, &cp);
    *wi = sinTheta * cp * v1 + sinTheta * sp * v2 + cosTheta * (-wo);
    return PhaseHG(-cosTheta, g);
}
static inline Float HG_p(Float g, const V3 &wo, const V3 &wi) { return PhaseHG(Dot(wo, wi), g); }

// ---- rays, scene ----
struct Ray {
    V3 o, d;
    Float tMax;
    V3 operator()(Float t) const { return o + d * t; }
};

// One pbrt Triangle (src/shapes/triangle.cpp) with the per-shape constants the passes use.
struct Tri {
    V3 p0, p1, p2;
    V3 n;       // Intersect's normal: Normalize(Cross(dp02, dp12)), negated if flip (:292-297)
    V3 ss, ts;  // BSDF frame: ss = Normalize(dpdu), ts = Cross(ns, ss) (reflection.h BSDF ctor)
    V3 nS;      // Sample's normal: Normalize(Cross(p1 - p0, p2 - p0)), negated if flip (:552-560)
    Float area;  // 0.5 * Cross(p1 - p0, p2 - p0).Length() (:535-541)
    Spectrum kd, Le;
    bool emit;
};

// Clamp, pbrt.h:278-284 (low first: Clamp(x, 0, -1) of a one-entry array is 0 for x < 0, else -1)
static inline int ClampInt(int val, int low, int high) {
    if (val < low) return low;
    if (val > high) return high;
    return val;
}
// FindInterval, pbrt.h:377-389: the largest index i in [0, size - 2] with pred(i) true (pred is
// monotone: true then false), by bisection; clamped to the first / last interval outside the range.
template <typename Predicate>
static inline int FindInterval(int size, const Predicate &pred) {
    int first = 0, len = size;
    while (len > 0) {
        int half = len >> 1, middle = first + half;
        if (pred(middle)) {
            first = middle + 1;
            len -= half + 1;
        } else {
            len = half;
        }
    }
    return ClampInt(first - 1, 0, size - 2);
}

// Distribution1D, sampling.h:55-100: the piecewise-constant CDF of func (the constructor) and
// SampleDiscrete with FindInterval (sampling.h:90-100, pbrt.h:377-389)
struct Distribution1D {
    std::vector<Float> func, cdf;
    Float funcInt = 0;
    Distribution1D() = default;
    Distribution1D(const Float *f, int n) : func(f, f + n), cdf(n + 1) {
        cdf[0] = 0;
        for (int i = 1; i < n + 1; ++i) cdf[i] = cdf[i - 1] + func[i - 1] / (Float)n;
        funcInt = cdf[n];
        if (funcInt == 0) {
            for (int i = 1; i < n + 1; ++i) cdf[i] = Float(i) / Float(n);
        } else {
            for (int i = 1; i < n + 1; ++i) cdf[i] /= funcInt;
        }
    }
    int Count() const { return (int)func.size(); }
    int SampleDiscrete(Float u, Float *pdf, Float *uRemapped = nullptr) const {
        const int offset = FindInterval((int)cdf.size(), [&](int i) { return cdf[i] <= u; });
        if (pdf) *pdf = (funcInt > 0) ? func[offset] / (funcInt * (Float)Count()) : 0;
        if (uRemapped) *uRemapped = (u - cdf[offset]) / (cdf[offset + 1] - cdf[offset]);
        return offset;
    }
    Float DiscretePDF(int index) const { return func[index] / (funcInt * (Float)Count()); }
    // SampleContinuous (sampling.h:71-89): the same FindInterval, then the offset along the segment
    Float SampleContinuous(Float u, Float *pdf, int *off = nullptr) const {
        const int offset = FindInterval((int)cdf.size(), [&](int i) { return cdf[i] <= u; });
        if (off) *off = offset;
        Float du = u - cdf[offset];
        if ((cdf[offset + 1] - cdf[offset]) > 0) du /= (cdf[offset + 1] - cdf[offset]);
        if (pdf) *pdf = (funcInt > 0) ? func[offset] / funcInt : 0;
        return (offset + du) / Count();
    }
};

// BVHAccel (src/accelerators/bvh.cpp): the scene's aggregate.  LinearBVHNode (bvh.cpp) in
// depth-first order: an interior node's first child follows it, the second is at secondChildOffset.
struct LinearBVHNode {
    V3 pMin, pMax;
    int offset;       // primitivesOffset (leaf) / secondChildOffset (interior)
    int nPrimitives;  // 0: interior
    int axis;
};

struct Scene {
    std::vector<Tri> tris;
    std::vector<LinearBVHNode> nodes;  // BVHAccel over tris (CreateBVHAccelerator defaults)
    std::vector<int> orderedPrims;     // BVHAccel::primitives after the build: triangle indices
    std::vector<int> lights;  // scene.lights: the emitting triangles, in triangle order
    // ComputeLightPowerDistribution (integrator.cpp:217-225) -> Distribution1D (sampling.h:55-100)
    Distribution1D ldist;
    bool medium;
    Spectrum sigma_t, sigma_s;
    Float g;
    // GridDensityMedium (grid.h:50-100)
    bool grid = false;
    int nx = 0, ny = 0, nz = 0;
    Float m[4][4];  // WorldToMedium
    const float *density = nullptr;
    Float gridSigmaT = 0, invMaxDensity = 0;
};

// the light-power distribution's SampleDiscrete (Distribution1D above)
static int SampleDiscrete(const Scene &sc, Float u, Float *pdf) { return sc.ldist.SampleDiscrete(u, pdf); }

// ---- BVHAccel (bvh.cpp), restated: recursiveBuild with SplitMethod::SAH, maxPrimsInNode 4 ----
struct Bounds3f {
    V3 pMin = V3(std::numeric_limits<Float>::max(), std::numeric_limits<Float>::max(),
                 std::numeric_limits<Float>::max());
    V3 pMax = V3(std::numeric_limits<Float>::lowest(), std::numeric_limits<Float>::lowest(),
                 std::numeric_limits<Float>::lowest());
    int MaximumExtent() const {
        const V3 d = pMax - pMin;
        if (d.x > d.y && d.x > d.z) return 0;
        else if (d.y > d.z) return 1;
        else return 2;
    }
    Float SurfaceArea() const {
        const V3 d = pMax - pMin;
        return 2 * (d.x * d.y + d.x * d.z + d.y * d.z);
    }
    V3 Offset(const V3 &p) const {
        V3 o = p - pMin;
        if (pMax.x > pMin.x) o.x /= pMax.x - pMin.x;
        if (pMax.y > pMin.y) o.y /= pMax.y - pMin.y;
        if (pMax.z > pMin.z) o.z /= pMax.z - pMin.z;
        return o;
    }
};
static inline Bounds3f Union(const Bounds3f &b, const V3 &p) {
    Bounds3f r;
    r.pMin = V3(std::min(b.pMin.x, p.x), std::min(b.pMin.y, p.y), std::min(b.pMin.z, p.z));
    r.pMax = V3(std::max(b.pMax.x, p.x), std::max(b.pMax.y, p.y), std::max(b.pMax.z, p.z));
    return r;
}
static inline Bounds3f Union(const Bounds3f &a, const Bounds3f &b) {
    Bounds3f r;
    r.pMin = V3(std::min(a.pMin.x, b.pMin.x), std::min(a.pMin.y, b.pMin.y), std::min(a.pMin.z, b.pMin.z));
    r.pMax = V3(std::max(a.pMax.x, b.pMax.x), std::max(a.pMax.y, b.pMax.y), std::max(a.pMax.z, b.pMax.z));
    return r;
}
struct BVHPrimitiveInfo {
    size_t primitiveNumber;
    Bounds3f bounds;
    V3 centroid;
};
struct BVHBuildNode {
    Bounds3f bounds;
    BVHBuildNode *children[2] = {nullptr, nullptr};
    int splitAxis = 0, firstPrimOffset = 0, nPrimitives = 0;
};
struct BVHBuilder {
    std::vector<BVHPrimitiveInfo> &info;
    std::vector<int> &orderedPrims;
    std::vector<std::unique_ptr<BVHBuildNode>> arena;
    int totalNodes = 0;
    BVHBuildNode *leaf(int start, int end, const Bounds3f &bounds) {
        BVHBuildNode *node = arena.back().get();
        node->firstPrimOffset = (int)orderedPrims.size();
        for (int i = start; i < end; ++i) orderedPrims.push_back((int)info[i].primitiveNumber);
        node->nPrimitives = end - start;
        node->bounds = bounds;
        return node;
    }
    BVHBuildNode *build(int start, int end) {  // recursiveBuild
        arena.emplace_back(new BVHBuildNode());
        BVHBuildNode *node = arena.back().get();
        ++totalNodes;
        Bounds3f bounds;
        for (int i = start; i < end; ++i) bounds = Union(bounds, info[i].bounds);
        const int nPrimitives = end - start;
        if (nPrimitives == 1) return leaf(start, end, bounds);
        Bounds3f centroidBounds;
        for (int i = start; i < end; ++i) centroidBounds = Union(centroidBounds, info[i].centroid);
        const int dim = centroidBounds.MaximumExtent();
        int mid = (start + end) / 2;
        if (centroidBounds.pMax[dim] == centroidBounds.pMin[dim]) return leaf(start, end, bounds);
        if (nPrimitives <= 2) {
            mid = (start + end) / 2;
            std::nth_element(&info[start], &info[mid], &info[end - 1] + 1,
                             [dim](const BVHPrimitiveInfo &a, const BVHPrimitiveInfo &b) {
                                 return a.centroid[dim] < b.centroid[dim];
                             });
        } else {
            const int nBuckets = 12;
            int count[12] = {};
            Bounds3f bb[12];
            for (int i = start; i < end; ++i) {
                int b = nBuckets * centroidBounds.Offset(info[i].centroid)[dim];
                if (b == nBuckets) b = nBuckets - 1;
                count[b]++;
                bb[b] = Union(bb[b], info[i].bounds);
            }
            Float cost[11];
            for (int i = 0; i < nBuckets - 1; ++i) {
                Bounds3f b0, b1;
                int count0 = 0, count1 = 0;
                for (int j = 0; j <= i; ++j) {
                    b0 = Union(b0, bb[j]);
                    count0 += count[j];
                }
                for (int j = i + 1; j < nBuckets; ++j) {
                    b1 = Union(b1, bb[j]);
                    count1 += count[j];
                }
                cost[i] = 1 + (count0 * b0.SurfaceArea() + count1 * b1.SurfaceArea()) / bounds.SurfaceArea();
            }
            Float minCost = cost[0];
            int minCostSplitBucket = 0;
            for (int i = 1; i < nBuckets - 1; ++i)
                if (cost[i] < minCost) {
                    minCost = cost[i];
                    minCostSplitBucket = i;
                }
            const Float leafCost = nPrimitives;
            const int maxPrimsInNode = 4;
            if (nPrimitives > maxPrimsInNode || minCost < leafCost) {
                BVHPrimitiveInfo *pmid = std::partition(&info[start], &info[end - 1] + 1, [=](const BVHPrimitiveInfo &pi) {
                    int b = nBuckets * centroidBounds.Offset(pi.centroid)[dim];
                    if (b == nBuckets) b = nBuckets - 1;
                    return b <= minCostSplitBucket;
                });
                mid = (int)(pmid - &info[0]);
            } else {
                return leaf(start, end, bounds);
            }
        }
        BVHBuildNode *c0 = build(start, mid);
        BVHBuildNode *c1 = build(mid, end);
        node->children[0] = c0;
        node->children[1] = c1;
        node->bounds = Union(c0->bounds, c1->bounds);  // InitInterior
        node->splitAxis = dim;
        node->nPrimitives = 0;
        return node;
    }
};
static int flattenBVHTree(const BVHBuildNode *node, std::vector<LinearBVHNode> &nodes) {  // flattenBVHTree
    const int myOffset = (int)nodes.size();
    nodes.push_back(LinearBVHNode{node->bounds.pMin, node->bounds.pMax, 0, node->nPrimitives, 0});
    if (node->nPrimitives > 0) {
        nodes[myOffset].offset = node->firstPrimOffset;
    } else {
        nodes[myOffset].axis = node->splitAxis;
        flattenBVHTree(node->children[0], nodes);
        nodes[myOffset].offset = flattenBVHTree(node->children[1], nodes);
    }
    return myOffset;
}
// BVHAccel ctor over the scene's triangles in order (Triangle::WorldBound: Union(Bounds3f(p0, p1), p2))
static void BuildSceneBVH(Scene &sc) {
    std::vector<BVHPrimitiveInfo> info(sc.tris.size());
    for (size_t i = 0; i < sc.tris.size(); ++i) {
        const Tri &T = sc.tris[i];
        Bounds3f b;
        b.pMin = V3(std::min(T.p0.x, T.p1.x), std::min(T.p0.y, T.p1.y), std::min(T.p0.z, T.p1.z));
        b.pMax = V3(std::max(T.p0.x, T.p1.x), std::max(T.p0.y, T.p1.y), std::max(T.p0.z, T.p1.z));
        b = Union(b, T.p2);
        info[i].primitiveNumber = i;
        info[i].bounds = b;
        info[i].centroid = b.pMin * .5f + b.pMax * .5f;  // .5f * pMin + .5f * pMax
    }
    sc.nodes.clear();
    sc.orderedPrims.clear();
    if (info.empty()) return;
    BVHBuilder bld{info, sc.orderedPrims, {}, 0};
    BVHBuildNode *root = bld.build(0, (int)info.size());
    flattenBVHTree(root, sc.nodes);
}

static Scene make_scene(const bre_scene *s) {
    Scene sc;
    const bre_triangle *tri = s->triangles_ext ? s->triangles_ext : s->triangles;
    for (int i = 0; i < s->n_triangles; ++i) {
        const bre_triangle &t = tri[i];
        Tri T;
        T.p0 = V3(t.p[0]);
        T.p1 = V3(t.p[1]);
        T.p2 = V3(t.p[2]);
        const V3 dp02 = T.p0 - T.p2, dp12 = T.p1 - T.p2;
        // dpdu for uvs (0,0), (1,0), (1,1): (duv12[1] * dp02 - duv02[1] * dp12) * invdet, with
        // duv12[1] = duv02[1] = -1 and invdet = 1 (triangle.cpp:276-285)
        const V3 dpdu = (dp02 * (Float)-1 - dp12 * (Float)-1) * (Float)1;
        T.n = Normalize(Cross(dp02, dp12));
        T.nS = Normalize(Cross(T.p1 - T.p0, T.p2 - T.p0));
        if (t.flip) {
            T.n = -T.n;
            T.nS = -T.nS;
        }
        T.ss = Normalize(dpdu);
        T.ts = Cross(T.n, T.ss);
        T.area = (Float)(0.5 * (double)Cross(T.p1 - T.p0, T.p2 - T.p0).Length());
        T.kd = Spectrum(t.kd);
        T.Le = Spectrum(t.Le);
        T.emit = t.emit != 0;
        if (T.emit) sc.lights.push_back(i);
        sc.tris.push_back(T);
    }
    // DiffuseAreaLight::Power() = (twoSided ? 2 : 1) * Lemit * area * Pi (diffuse.cpp:53-55), .y()
    std::vector<Float> lfunc;
    for (int l : sc.lights) {
        const Tri &T = sc.tris[l];
        lfunc.push_back(((T.Le * (Float)1) * T.area * Pi).y());
    }
    if (!lfunc.empty()) sc.ldist = Distribution1D(lfunc.data(), (int)lfunc.size());
    BuildSceneBVH(sc);
    sc.medium = s->has_medium != 0;
    Spectrum sa(s->sigma_a);
    sc.sigma_s = Spectrum(s->sigma_s);
    sc.sigma_t = sa + sc.sigma_s;
    sc.g = s->g;
    if (s->has_medium == BRE_MEDIUM_GRID) {
        sc.grid = true;
        sc.nx = s->grid_n[0];
        sc.ny = s->grid_n[1];
        sc.nz = s->grid_n[2];
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) sc.m[i][j] = s->world_to_medium[4 * i + j];
        sc.density = s->grid_density;
        sc.gridSigmaT = (sa + sc.sigma_s).c[0];
        Float maxDensity = 0;
        for (int i = 0; i < sc.nx * sc.ny * sc.nz; ++i) maxDensity = std::max(maxDensity, sc.density[i]);
        sc.invMaxDensity = 1 / maxDensity;
    }
    return sc;
}

struct Isect {
    V3 p, pError, n;
    int tri = -1;
};

static inline int MaxDimension(const V3 &v) { return (v.x > v.y) ? ((v.x > v.z) ? 0 : 2) : ((v.y > v.z) ? 1 : 2); }
static inline V3 Permute(const V3 &v, int x, int y, int z) { return V3(v[x], v[y], v[z]); }
static inline Float MaxComponent(const V3 &v) { return std::max(v.x, std::max(v.y, v.z)); }

// Triangle::Intersect, triangle.cpp:177-300 (watertight ray-triangle test; no alpha texture)
static bool IntersectTri(const Tri &T, const Ray &ray, Float *tHit, Isect *isect) {
    const V3 &p0 = T.p0, &p1 = T.p1, &p2 = T.p2;
    V3 p0t = p0 - ray.o, p1t = p1 - ray.o, p2t = p2 - ray.o;
    int kz = MaxDimension(Abs(ray.d));
    int kx = kz + 1;
    if (kx == 3) kx = 0;
    int ky = kx + 1;
    if (ky == 3) ky = 0;
    V3 d = Permute(ray.d, kx, ky, kz);
    p0t = Permute(p0t, kx, ky, kz);
    p1t = Permute(p1t, kx, ky, kz);
    p2t = Permute(p2t, kx, ky, kz);
    Float Sx = -d.x / d.z;
    Float Sy = -d.y / d.z;
    Float Sz = 1.f / d.z;
    p0t.x += Sx * p0t.z;
    p0t.y += Sy * p0t.z;
    p1t.x += Sx * p1t.z;
    p1t.y += Sy * p1t.z;
    p2t.x += Sx * p2t.z;
    p2t.y += Sy * p2t.z;
    Float e0 = p1t.x * p2t.y - p1t.y * p2t.x;
    Float e1 = p2t.x * p0t.y - p2t.y * p0t.x;
    Float e2 = p0t.x * p1t.y - p0t.y * p1t.x;
    if (e0 == 0.0f || e1 == 0.0f || e2 == 0.0f) {
        double p2txp1ty = (double)p2t.x * (double)p1t.y;
        double p2typ1tx = (double)p2t.y * (double)p1t.x;
        e0 = (float)(p2typ1tx - p2txp1ty);
        double p0txp2ty = (double)p0t.x * (double)p2t.y;
        double p0typ2tx = (double)p0t.y * (double)p2t.x;
        e1 = (float)(p0typ2tx - p0txp2ty);
        double p1txp0ty = (double)p1t.x * (double)p0t.y;
        double p1typ0tx = (double)p1t.y * (double)p0t.x;
        e2 = (float)(p1typ0tx - p1txp0ty);
    }
    if ((e0 < 0 || e1 < 0 || e2 < 0) && (e0 > 0 || e1 > 0 || e2 > 0)) return false;
    Float det = e0 + e1 + e2;
    if (det == 0) return false;
    p0t.z *= Sz;
    p1t.z *= Sz;
    p2t.z *= Sz;
    Float tScaled = e0 * p0t.z + e1 * p1t.z + e2 * p2t.z;
    if (det < 0 && (tScaled >= 0 || tScaled < ray.tMax * det)) return false;
    else if (det > 0 && (tScaled <= 0 || tScaled > ray.tMax * det)) return false;
    Float invDet = 1 / det;
    Float b0 = e0 * invDet;
    Float b1 = e1 * invDet;
    Float b2 = e2 * invDet;
    Float t = tScaled * invDet;
    Float maxZt = MaxComponent(Abs(V3(p0t.z, p1t.z, p2t.z)));
    Float deltaZ = gamma(3) * maxZt;
    Float maxXt = MaxComponent(Abs(V3(p0t.x, p1t.x, p2t.x)));
    Float maxYt = MaxComponent(Abs(V3(p0t.y, p1t.y, p2t.y)));
    Float deltaX = gamma(5) * (maxXt + maxZt);
    Float deltaY = gamma(5) * (maxYt + maxZt);
    Float deltaE = 2 * (gamma(2) * maxXt * maxYt + deltaY * maxXt + deltaX * maxYt);
    Float maxE = MaxComponent(Abs(V3(e0, e1, e2)));
    Float deltaT = 3 * (gamma(3) * maxE * maxZt + deltaE * maxZt + deltaZ * maxE) * std::abs(invDet);
    if (t <= deltaT) return false;
    Float xAbsSum = (std::abs(b0 * p0.x) + std::abs(b1 * p1.x) + std::abs(b2 * p2.x));
    Float yAbsSum = (std::abs(b0 * p0.y) + std::abs(b1 * p1.y) + std::abs(b2 * p2.y));
    Float zAbsSum = (std::abs(b0 * p0.z) + std::abs(b1 * p1.z) + std::abs(b2 * p2.z));
    isect->pError = V3(xAbsSum, yAbsSum, zAbsSum) * gamma(7);
    isect->p = p0 * b0 + p1 * b1 + p2 * b2;
    isect->n = T.n;
    *tHit = t;
    return true;
}

// Bounds3::IntersectP(ray, invDir, dirIsNeg), geometry.h:1410-1436
static inline bool IntersectP(const LinearBVHNode &b, const Ray &ray, const V3 &invDir, const int dirIsNeg[3]) {
    const V3 bnd[2] = {b.pMin, b.pMax};
    Float tMin = (bnd[dirIsNeg[0]].x - ray.o.x) * invDir.x;
    Float tMax = (bnd[1 - dirIsNeg[0]].x - ray.o.x) * invDir.x;
    Float tyMin = (bnd[dirIsNeg[1]].y - ray.o.y) * invDir.y;
    Float tyMax = (bnd[1 - dirIsNeg[1]].y - ray.o.y) * invDir.y;
    tMax *= 1 + 2 * gamma(3);
    tyMax *= 1 + 2 * gamma(3);
    if (tMin > tyMax || tyMin > tMax) return false;
    if (tyMin > tMin) tMin = tyMin;
    if (tyMax < tMax) tMax = tyMax;
    Float tzMin = (bnd[dirIsNeg[2]].z - ray.o.z) * invDir.z;
    Float tzMax = (bnd[1 - dirIsNeg[2]].z - ray.o.z) * invDir.z;
    tzMax *= 1 + 2 * gamma(3);
    if (tMin > tzMax || tzMin > tMax) return false;
    if (tzMin > tMin) tMin = tzMin;
    if (tzMax < tMax) tMax = tzMax;
    return (tMin < ray.tMax) && (tMax > 0);
}

// Scene::Intersect = BVHAccel::Intersect (bvh.cpp): depth first, near child first by dirIsNeg[axis];
// every hit shrinks ray.tMax (GeometricPrimitive::Intersect, primitive.cpp:97-101), so an
// equal-distance tie goes to the triangle the reference tests last.
static bool Intersect(const Scene &sc, Ray &ray, Isect *isect) {
    if (sc.nodes.empty()) return false;
    bool hit = false;
    const V3 invDir(1 / ray.d.x, 1 / ray.d.y, 1 / ray.d.z);
    const int dirIsNeg[3] = {invDir.x < 0, invDir.y < 0, invDir.z < 0};
    int toVisitOffset = 0, currentNodeIndex = 0;
    int nodesToVisit[64];
    while (true) {
        const LinearBVHNode *node = &sc.nodes[currentNodeIndex];
        if (IntersectP(*node, ray, invDir, dirIsNeg)) {
            if (node->nPrimitives > 0) {
                for (int i = 0; i < node->nPrimitives; ++i) {
                    const int ti = sc.orderedPrims[node->offset + i];
                    Float t;
                    Isect tmp;
                    if (!IntersectTri(sc.tris[ti], ray, &t, &tmp)) continue;
                    ray.tMax = t;
                    *isect = tmp;
                    isect->tri = ti;
                    hit = true;
                }
                if (toVisitOffset == 0) break;
                currentNodeIndex = nodesToVisit[--toVisitOffset];
            } else {
                if (dirIsNeg[node->axis]) {
                    nodesToVisit[toVisitOffset++] = currentNodeIndex + 1;
                    currentNodeIndex = node->offset;
                } else {
                    nodesToVisit[toVisitOffset++] = node->offset;
                    currentNodeIndex = currentNodeIndex + 1;
                }
            }
        } else {
            if (toVisitOffset == 0) break;
            currentNodeIndex = nodesToVisit[--toVisitOffset];
        }
    }
    return hit;
}

// The round-2 restatement (every triangle in scene order; a later triangle wins an exact tie):
// kept for tests/refpy_photon.py's independent cross-check.
static bool IntersectLinear(const Scene &sc, Ray &ray, Isect *isect) {
    bool hit = false;
    for (int i = 0; i < (int)sc.tris.size(); ++i) {
        Float t;
        Isect tmp;
        if (!IntersectTri(sc.tris[i], ray, &t, &tmp)) continue;
        ray.tMax = t;
        *isect = tmp;
        isect->tri = i;
        hit = true;
    }
    return hit;
}

// Triangle::Sample(u, pdf) (triangle.cpp:543-568) with UniformSampleTriangle (sampling.cpp)
struct ShapeSample {
    V3 p, pError, n;
    Float pdf;
};
static ShapeSample SampleTri(const Tri &T, Float u0, Float u1) {
    ShapeSample r;
    const Float su0 = std::sqrt(u0);
    const Float b0 = 1 - su0, b1 = u1 * su0;
    const Float b2 = 1 - b0 - b1;
    r.p = T.p0 * b0 + T.p1 * b1 + T.p2 * b2;
    r.n = T.nS;
    const V3 pAbsSum = Abs(T.p0 * b0) + Abs(T.p1 * b1) + Abs(T.p2 * b2);
    r.pError = pAbsSum * gamma(6);
    r.pdf = 1 / T.area;
    return r;
}

// HomogeneousMedium (homogeneous.cpp:44-77)
static Spectrum HomogeneousTr(const Scene &sc, const Ray &ray) {
    return Exp(-sc.sigma_t * std::min(ray.tMax * ray.d.Length(), MaxFloat));
}
// returns sampledMedium; *t = sampled distance.  (The returned weight is unused by the photon
// tracer, which overwrites betaMedium with Tr, photonbeam.cpp:289.)
template <class S>
static bool HomogeneousSample(const Scene &sc, const Ray &ray, S &sampler, Float *tOut) {
    int channel = std::min((int)(sampler.Get1D() * 3), 3 - 1);
    Float dist = -ora_log(1 - sampler.Get1D()) / sc.sigma_t.c[channel];
    Float t = std::min(dist * ray.d.Length(), ray.tMax);
    *tOut = t;
    return t < ray.tMax;
}

// ---- GridDensityMedium (grid.h:84-88, grid.cpp:46-118) ----
static inline Float Lerp(Float t, Float v1, Float v2) { return (1 - t) * v1 + t * v2; }
static Float GridD(const Scene &sc, int x, int y, int z) {
    // InsideExclusive(p, Bounds3i((0,0,0), (nx,ny,nz)))
    if (!(x >= 0 && x < sc.nx && y >= 0 && y < sc.ny && z >= 0 && z < sc.nz)) return 0;
    return sc.density[(z * sc.ny + y) * sc.nx + x];
}
static Float GridDensity(const Scene &sc, const V3 &p) {
    V3 ps(p.x * sc.nx - .5f, p.y * sc.ny - .5f, p.z * sc.nz - .5f);
    int pi[3] = {(int)std::floor(ps.x), (int)std::floor(ps.y), (int)std::floor(ps.z)};
    V3 d(ps.x - (Float)pi[0], ps.y - (Float)pi[1], ps.z - (Float)pi[2]);
    Float d00 = Lerp(d.x, GridD(sc, pi[0], pi[1], pi[2]), GridD(sc, pi[0] + 1, pi[1], pi[2]));
    Float d10 = Lerp(d.x, GridD(sc, pi[0], pi[1] + 1, pi[2]), GridD(sc, pi[0] + 1, pi[1] + 1, pi[2]));
    Float d01 = Lerp(d.x, GridD(sc, pi[0], pi[1], pi[2] + 1), GridD(sc, pi[0] + 1, pi[1], pi[2] + 1));
    Float d11 = Lerp(d.x, GridD(sc, pi[0], pi[1] + 1, pi[2] + 1), GridD(sc, pi[0] + 1, pi[1] + 1, pi[2] + 1));
    Float d0 = Lerp(d.y, d00, d10);
    Float d1 = Lerp(d.y, d01, d11);
    return Lerp(d.z, d0, d1);
}
// Transform::operator()(const Ray &) (transform.h:251-264) with the point transform and its error
// bound (:278-299) and the vector transform (:236-242)
static Ray TransformRay(const Float m[4][4], const Ray &r) {
    Float x = r.o.x, y = r.o.y, z = r.o.z;
    Float xp = m[0][0] * x + m[0][1] * y + m[0][2] * z + m[0][3];
    Float yp = m[1][0] * x + m[1][1] * y + m[1][2] * z + m[1][3];
    Float zp = m[2][0] * x + m[2][1] * y + m[2][2] * z + m[2][3];
    Float wp = m[3][0] * x + m[3][1] * y + m[3][2] * z + m[3][3];
    Float xAbsSum = (std::abs(m[0][0] * x) + std::abs(m[0][1] * y) + std::abs(m[0][2] * z) + std::abs(m[0][3]));
    Float yAbsSum = (std::abs(m[1][0] * x) + std::abs(m[1][1] * y) + std::abs(m[1][2] * z) + std::abs(m[1][3]));
    Float zAbsSum = (std::abs(m[2][0] * x) + std::abs(m[2][1] * y) + std::abs(m[2][2] * z) + std::abs(m[2][3]));
    V3 oError = V3(xAbsSum, yAbsSum, zAbsSum) * gamma(3);
    V3 o = (wp == 1) ? V3(xp, yp, zp) : V3(xp, yp, zp) * ((Float)1 / wp);
    V3 d(m[0][0] * r.d.x + m[0][1] * r.d.y + m[0][2] * r.d.z, m[1][0] * r.d.x + m[1][1] * r.d.y + m[1][2] * r.d.z,
         m[2][0] * r.d.x + m[2][1] * r.d.y + m[2][2] * r.d.z);
    Float lengthSquared = d.LengthSquared();
    Float tMax = r.tMax;
    if (lengthSquared > 0) {
        Float dt = Dot(Abs(d), oError) / lengthSquared;
        o = o + d * dt;
        tMax -= dt;
    }
    Ray out;
    out.o = o;
    out.d = d;
    out.tMax = tMax;
    return out;
}
// Bounds3f((0,0,0), (1,1,1)).IntersectP(ray, &t0, &t1), geometry.h:1386-1408
static bool UnitBoxIntersectP(const Ray &ray, Float *hitt0, Float *hitt1) {
    Float t0 = 0, t1 = ray.tMax;
    for (int i = 0; i < 3; ++i) {
        Float invRayDir = 1 / ray.d[i];
        Float tNear = ((Float)0 - ray.o[i]) * invRayDir;
        Float tFar = ((Float)1 - ray.o[i]) * invRayDir;
        if (tNear > tFar) std::swap(tNear, tFar);
        tFar *= 1 + 2 * gamma(3);
        t0 = tNear > t0 ? tNear : t0;
        t1 = tFar < t1 ? tFar : t1;
        if (t0 > t1) return false;
    }
    *hitt0 = t0;
    *hitt1 = t1;
    return true;
}
static Ray GridMediumRay(const Scene &sc, const Ray &rWorld) {
    Ray r;
    r.o = rWorld.o;
    r.d = Normalize(rWorld.d);
    r.tMax = rWorld.tMax * rWorld.d.Length();
    return TransformRay(sc.m, r);
}
// GridDensityMedium::Sample (grid.cpp:62-89): delta tracking; the interaction is at rWorld(t)
template <class S>
static bool GridSample(const Scene &sc, const Ray &rWorld, S &sampler, Float *tOut) {
    Ray ray = GridMediumRay(sc, rWorld);
    Float tMin, tMax;
    if (!UnitBoxIntersectP(ray, &tMin, &tMax)) return false;
    Float t = tMin;
    while (true) {
        t -= ora_log(1 - sampler.Get1D()) * sc.invMaxDensity / sc.gridSigmaT;
        if (t >= tMax) break;
        if (GridDensity(sc, ray(t)) * sc.invMaxDensity > sampler.Get1D()) {
            *tOut = t;
            return true;
        }
    }
    return false;
}
// GridDensityMedium::Tr (grid.cpp:91-118): ratio tracking with Russian roulette below 0.1
template <class S>
static Spectrum GridTr(const Scene &sc, const Ray &rWorld, S &sampler) {
    Ray ray = GridMediumRay(sc, rWorld);
    Float tMin, tMax;
    if (!UnitBoxIntersectP(ray, &tMin, &tMax)) return Spectrum(1.f);
    Float Tr = 1, t = tMin;
    while (true) {
        t -= ora_log(1 - sampler.Get1D()) * sc.invMaxDensity / sc.gridSigmaT;
        if (t >= tMax) break;
        Float density = GridDensity(sc, ray(t));
        Tr *= 1 - std::max((Float)0, density * sc.invMaxDensity);
        const Float rrThreshold = .1;
        if (Tr < rrThreshold) {
            Float q = std::max((Float).05, 1 - Tr);
            if (sampler.Get1D() < q) return Spectrum(0.f);
            Tr /= 1 - q;
        }
    }
    return Spectrum(Tr);
}

// Medium::Tr / Medium::Sample of the scene's medium
template <class S>
static Spectrum MediumTr(const Scene &sc, const Ray &ray, S &sampler) {
    return sc.grid ? GridTr(sc, ray, sampler) : HomogeneousTr(sc, ray);
}
template <class S>
static bool MediumSample(const Scene &sc, const Ray &ray, S &sampler, Float *tOut) {
    return sc.grid ? GridSample(sc, ray, sampler, tOut) : HomogeneousSample(sc, ray, sampler, tOut);
}

}  // namespace orp
