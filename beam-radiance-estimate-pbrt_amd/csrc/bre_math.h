// bre_math.h — float arithmetic of the reference's gather path, written for gfx950 device code.
//
// Every function reproduces the reference's operation order and precision so that one
// (segment, beam) pair gives bit-identical results to pbrt's x86-64 float code:
//   * no FMA contraction: this header must be compiled with -ffp-contract=off (csrc/Makefile);
//   * correctly rounded division and sqrt (-fhip-fp32-correctly-rounded-divide-sqrt);
//   * Vector3 operator/ multiplies by (Float)1/f  (geometry.h:244-257);
//   * Cross is evaluated in double and rounded to float (geometry.h:957-963);
//   * std::min / std::max NaN behaviour is kept where it matters (Bounds3 ctor, geometry.h:759-763).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bre {

struct f3 {
    float x, y, z;
};

__host__ __device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__host__ __device__ __forceinline__ f3 add3(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__host__ __device__ __forceinline__ f3 sub3(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
// Vector3::operator*(U s) = (s*x, s*y, s*z)
__host__ __device__ __forceinline__ f3 scale3(f3 a, float s) { return mk(s * a.x, s * a.y, s * a.z); }
// Vector3::operator/(U f): inv = 1/f, then multiply
__host__ __device__ __forceinline__ f3 div3(f3 a, float f) {
    const float inv = 1.0f / f;
    return mk(a.x * inv, a.y * inv, a.z * inv);
}
__host__ __device__ __forceinline__ float dot3(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__host__ __device__ __forceinline__ float lensq3(f3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
__host__ __device__ __forceinline__ float len3(f3 a) { return sqrtf(lensq3(a)); }

// Cross(v1, v2) in double, geometry.h:957-963.  A product of two floats is exact in double (24 + 24
// significant bits <= 53), so (a*b) - (c*d) with both products rounded is fma(a, b, -(c*d)): the same
// single rounding of the exact difference, one double instruction less per component.
__host__ __device__ __forceinline__ f3 cross3d(f3 v1, f3 v2) {
    const double v1x = v1.x, v1y = v1.y, v1z = v1.z;
    const double v2x = v2.x, v2y = v2.y, v2z = v2.z;
    return mk((float)__builtin_fma(v1y, v2z, -(v1z * v2y)), (float)__builtin_fma(v1z, v2x, -(v1x * v2z)),
              (float)__builtin_fma(v1x, v2y, -(v1y * v2x)));
}

// Determinant, photonbeam.cpp:79-85
__host__ __device__ __forceinline__ float det3(f3 a, f3 b, f3 c) {
    return a.x * b.y * c.z + a.y * b.z * c.x + a.z * b.x * c.y - (a.z * b.y * c.x + a.y * b.x * c.z + a.x * b.z * c.y);
}

__host__ __device__ __forceinline__ float clampf_ref(float v, float lo, float hi) {  // pbrt.h:278-284
    return (v < lo) ? lo : ((v > hi) ? hi : v);
}
__host__ __device__ __forceinline__ float smin(float a, float b) { return (b < a) ? b : a; }  // std::min
__host__ __device__ __forceinline__ float smax(float a, float b) { return (a < b) ? b : a; }  // std::max

// 1 + 2*gamma(3) with MachineEpsilon = FLT_EPSILON/2, evaluated in float as pbrt does
// (pbrt.h:175-176, 263-265; geometry.h:1421).
__host__ __device__ __forceinline__ float slab_pad() {
    const float eps = 5.96046447753906250e-08f;  // 2^-24
    const float g3 = (3 * eps) / (1 - 3 * eps);
    return 1 + 2 * g3;
}

// PhotonBeam::WorldBound, photonbeambvh.h:60-72.  sqrt_mode 0: `sqrt` resolves to
// ::sqrt(double) under libstdc++, so `2*radius*sqrt(..)` and the `+` are double.
__host__ __device__ __forceinline__ void world_bound(f3 start, f3 end, float radius, int sqrt_mode, f3 &lo, f3 &hi) {
    f3 dir = sub3(end, start);
    const f3 center = add3(start, div3(dir, 2.0f));
    const float len = len3(dir);
    dir = div3(dir, len);
    f3 size;
    const float tr = 2 * radius;
    if (sqrt_mode == 0) {
        size.x = (float)((double)(dir.x * len) + (double)tr * sqrt((double)(1 - dir.x * dir.x)));
        size.y = (float)((double)(dir.y * len) + (double)tr * sqrt((double)(1 - dir.y * dir.y)));
        size.z = (float)((double)(dir.z * len) + (double)tr * sqrt((double)(1 - dir.z * dir.z)));
    } else {
        size.x = dir.x * len + tr * sqrtf(1 - dir.x * dir.x);
        size.y = dir.y * len + tr * sqrtf(1 - dir.y * dir.y);
        size.z = dir.z * len + tr * sqrtf(1 - dir.z * dir.z);
    }
    const f3 half = div3(size, 2.0f);
    const f3 p1 = sub3(center, half), p2 = add3(center, half);
    lo = mk(smin(p1.x, p2.x), smin(p1.y, p2.y), smin(p1.z, p2.z));
    hi = mk(smax(p1.x, p2.x), smax(p1.y, p2.y), smax(p1.z, p2.z));
}

// Bounds3::IntersectP(ray, invDir, dirIsNeg), geometry.h:1410-1436.  `inv` selects which inverse
// direction is used: the exact one reproduces the reference test; the sanitised one gives a test
// that is monotone under box containment (used for BVH interior nodes, which are unions).
// Box coordinates are passed by value so that wave-uniform boxes stay in SGPRs and the per-lane
// dirIsNeg choice is a register select, not a per-lane address.
struct Box6 {
    float lx, ly, lz, hx, hy, hz;
};
__host__ __device__ __forceinline__ bool slab_test(const Box6 &b, f3 o, f3 inv, int n0, int n1, int n2, float ray_tmax,
                                                   float *t_entry) {
    // Branch-free statement of the reference's sequence: every step is computed and the early
    // returns become a conjunction.  The `if (a > b) x = a` updates stay compare+select (not
    // fmaxf/fminf) so NaNs from 0*inf propagate exactly as in the reference.
    const float pad = slab_pad();
    float tMin = ((n0 ? b.hx : b.lx) - o.x) * inv.x;
    float tMax = ((n0 ? b.lx : b.hx) - o.x) * inv.x;
    const float tyMin = ((n1 ? b.hy : b.ly) - o.y) * inv.y;
    float tyMax = ((n1 ? b.ly : b.hy) - o.y) * inv.y;
    tMax *= pad;
    tyMax *= pad;
    const bool ok1 = !(tMin > tyMax || tyMin > tMax);
    tMin = (tyMin > tMin) ? tyMin : tMin;
    tMax = (tyMax < tMax) ? tyMax : tMax;
    const float tzMin = ((n2 ? b.hz : b.lz) - o.z) * inv.z;
    float tzMax = ((n2 ? b.lz : b.hz) - o.z) * inv.z;
    tzMax *= pad;
    const bool ok2 = !(tMin > tzMax || tzMin > tMax);
    tMin = (tzMin > tMin) ? tzMin : tMin;
    tMax = (tzMax < tMax) ? tzMax : tMax;
    if (t_entry) *t_entry = tMin;
    return ok1 & ok2 & (tMin < ray_tmax) & (tMax > 0);
}

// The same decision for a NaN-free inverse direction (|inv| finite, nonzero: the sanitised one),
// in min/max form: near/far per axis are min/max of the two plane distances (equal to the
// reference's dirIsNeg selection when inv is finite), the pairwise overlap tests collapse to
// max(near) <= min(far) (the self pairs hold whenever min(far) > 0), and the gamma(3) pad
// commutes with min because rounding is monotone.  Bit-identical decision to slab_test(b, invs),
// and monotone under box containment, so it is conservative for BVH interior (union) boxes.
__host__ __device__ __forceinline__ bool node_test(const Box6 &b, f3 o, f3 invs, float ray_tmax, float &t_entry) {
    const float ax = (b.lx - o.x) * invs.x, bx = (b.hx - o.x) * invs.x;
    const float ay = (b.ly - o.y) * invs.y, by = (b.hy - o.y) * invs.y;
    const float az = (b.lz - o.z) * invs.z, bz = (b.hz - o.z) * invs.z;
    const float tn = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
    const float tf = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz)) * slab_pad();
    t_entry = tn;
    return (tn <= tf) & (tn < ray_tmax) & (tf > 0);
}

// ComputeClosestPoints, photonbeam.cpp:87-186, specialised to precomputed unit directions:
//   segment A: a0, a1, au = (a1-a0)*(1/|A|), mag_a = |a1-a0|
//   beam    B: b0, bu = (b1-b0)*(1/|B|), mag_b = |b1-b0| (> 0: zero-length beams have a NaN
//              WorldBound and never become candidates, so the magB==0 branch is unreachable)
// Returns false for parallel lines (no contribution).  Writes |aClosest - bClosest|.
// With WANT_S, also returns the beam-line parameter s of the returned beam point, pB = b0 + bu*s
// (t1 when t0 is inside A, else the clamped projection of A's endpoint): the capsule-chunk
// index (bre_chunk.hip) assigns each pair to the chunk whose ownership interval holds s.
// SQ: return the squared distance lensq3(aClosest - bClosest) instead of its square root (the caller
// takes the correctly rounded root itself, e.g. sqrt_cr_noscale).
template <bool WANT_S, bool SQ = false>
__host__ __device__ __forceinline__ bool closest_distance_t(f3 a0, f3 a1, f3 au, float mag_a, f3 b0, f3 bu,
                                                            float mag_b, float &dist, float &s_out) {
    if (mag_a == 0.0f) {
        // A is a point: project a0 onto B, clamp (photonbeam.cpp:95-108)
        const float d = dot3(sub3(a0, b0), bu);
        const float dc = clampf_ref(d, 0.0f, mag_b);
        const f3 bc = add3(b0, scale3(bu, dc));
        dist = SQ ? lensq3(sub3(a0, bc)) : len3(sub3(a0, bc));
        if (WANT_S) s_out = dc;
        return true;
    }
    const f3 cr = cross3d(au, bu);
    const float denom = lensq3(cr);
    if (denom == 0.0f) return false;  // parallel (photonbeam.cpp:131-156)
    const f3 t = sub3(b0, a0);
    const float detA = det3(t, bu, cr);
    const float detB = det3(t, au, cr);
    const float t0 = detA / denom;
    const float t1 = detB / denom;
    f3 pA = add3(a0, scale3(au, t0));
    f3 pB = add3(b0, scale3(bu, t1));
    float sb = t1;
    if (t0 < 0) pA = a0;
    else if (t0 > mag_a) pA = a1;
    if (t0 < 0 || t0 > mag_a) {
        const float d = clampf_ref(dot3(bu, sub3(pA, b0)), 0.0f, mag_b);
        pB = add3(b0, scale3(bu, d));
        sb = d;
    }
    if (t1 < 0 || t1 > mag_b) {
        const float d = clampf_ref(dot3(au, sub3(pB, a0)), 0.0f, mag_a);
        pA = add3(a0, scale3(au, d));
    }
    dist = SQ ? lensq3(sub3(pA, pB)) : len3(sub3(pA, pB));
    if (WANT_S) s_out = sb;
    return true;
}

// The correctly rounded float square root without the small-input scaling of the compiler's
// expansion: v_sqrt_f32 (within 1 ulp) and the same +-1 ulp residual correction, in the same order.
// For x >= 2^-96 the compiler's sequence takes exactly these steps, so the result is bit-identical
// to sqrtf(x) there; also for 0, +inf and NaN (as NaN).  Below 2^-96 (the compiler scales by 2^32
// first) the result may differ in the last bits: callers use it only where such inputs cannot occur
// or cannot change a result.
__device__ __forceinline__ float sqrt_cr_noscale(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __int_as_float(__float_as_int(s) - 1);
    const float sp = __int_as_float(__float_as_int(s) + 1);
    const float rm = __builtin_fmaf(-sm, s, x);
    const float rp = __builtin_fmaf(-sp, s, x);
    const float r = (rm <= 0.0f) ? sm : s;
    return (rp > 0.0f) ? sp : r;
}

// a / b correctly rounded for a divisor b shared by many divisions, given y = 1 / b correctly rounded
// (computed once): q0 = a y, then two Markstein corrections r = a - b q (exact by FMA), q + r y.  After
// the first, q is a faithful quotient; with y within half an ulp of 1 / b, the second then returns
// RN(a / b) (Markstein's theorem; Muller et al., Handbook of Floating-Point Arithmetic, the division
// chapter), barring underflow / overflow.  Five VALU instead of the general expansion's ten plus its
// scaling steps.  Callers: a, b finite, b > 0, a / b not below the normal range or where such a
// quotient cannot change the result.
__device__ __forceinline__ float div_by_shared(float a, float b, float y) {
    const float q0 = a * y;
    const float r0 = __builtin_fmaf(-q0, b, a);
    const float q1 = __builtin_fmaf(r0, y, q0);
    const float r1 = __builtin_fmaf(-q1, b, a);
    return __builtin_fmaf(r1, y, q1);
}

__host__ __device__ __forceinline__ bool closest_distance(f3 a0, f3 a1, f3 au, float mag_a, f3 b0, f3 bu, float mag_b,
                                                          float &dist) {
    float unused;
    return closest_distance_t<false>(a0, a1, au, mag_a, b0, bu, mag_b, dist, unused);
}

// Hilbert curve index of an n-dimensional point with b bits per coordinate (Skilling, "Programming
// the Hilbert curve", AIP Conf. Proc. 707, 2004: AxestoTranspose, then the bits interleaved from the
// most significant down).  A Hilbert order has no long jumps between consecutive cells, unlike a
// Morton order, so runs of consecutive keys (leaf tiles, segment packets) are more compact.
template <int N, int B>
__host__ __device__ __forceinline__ unsigned long long hilbert_key(unsigned int x[N]) {
    const unsigned int M = 1u << (B - 1);
    for (unsigned int Q = M; Q > 1; Q >>= 1) {  // inverse undo
        const unsigned int P = Q - 1;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            if (x[i] & Q) {
                x[0] ^= P;  // invert
            } else {        // exchange
                const unsigned int t = (x[0] ^ x[i]) & P;
                x[0] ^= t;
                x[i] ^= t;
            }
        }
    }
#pragma unroll
    for (int i = 1; i < N; ++i) x[i] ^= x[i - 1];  // Gray encode
    unsigned int t = 0;
    for (unsigned int Q = M; Q > 1; Q >>= 1)
        if (x[N - 1] & Q) t ^= Q - 1;
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] ^= t;
    unsigned long long key = 0ull;
    for (int bit = B - 1; bit >= 0; --bit)
#pragma unroll
        for (int i = 0; i < N; ++i) key = (key << 1) | ((x[i] >> bit) & 1u);
    return key;
}

}  // namespace bre
