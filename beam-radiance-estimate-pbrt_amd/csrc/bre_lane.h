// bre_lane.h — per-lane segment state and the record loads / conservative tests shared by the
// gather kernels (bre_gather.hip: reference candidate enumeration; bre_chunk.hip: capsule-chunk
// index).  Device code only; compiled with -ffp-contract=off (csrc/Makefile).
#pragma once

#include <hip/hip_runtime.h>

#include <float.h>

#include "bre_device.h"
#include "bre_math.h"

namespace bre {
namespace {

// Whole-record loads (4 x 16 B).  With a wave-uniform index these become SMEM loads into SGPRs.
struct NodeV {
    Box6 b0, b1;
    int32_t c0, c1;
};
__device__ __forceinline__ NodeV load_node(const Node *__restrict__ nodes, int i) {
    const float4 *q = reinterpret_cast<const float4 *>(nodes + i);
    const float4 x = q[0], y = q[1], z = q[2], w = q[3];
    NodeV n;
    // Node layout: lo[0] (0-2), lo[1] (3-5), hi[0] (6-8), hi[1] (9-11), child[0], child[1], ...
    n.b0 = Box6{x.x, x.y, x.z, y.z, y.w, z.x};
    n.b1 = Box6{x.w, y.x, y.y, z.y, z.z, z.w};
    n.c0 = __float_as_int(w.x);
    n.c1 = __float_as_int(w.y);
    return n;
}
struct BeamV {
    Box6 box;
    f3 b0, bu;
    float mag_b, radius;
    f3 pw;  // scaled powerEnd, when the caller already has it (kernel 3 batches)
};
__device__ __forceinline__ BeamV load_beam(const BeamRec *__restrict__ recs, int64_t i, const BeamSet &bs) {
    const float4 *q = reinterpret_cast<const float4 *>(recs + i);
    const float4 x = q[0], y = q[1], z = q[2], w = q[3];
    BeamV r;
    r.box = Box6{x.x, x.y, x.z, x.w, y.x, y.y};
    r.b0 = mk(y.z, y.w, z.x);
    r.bu = mk(z.y, z.z, z.w);
    r.mag_b = w.x;
    r.radius = beam_radius(bs, w.y);
    r.pw = mk(0.f, 0.f, 0.f);
    return r;
}

struct Lane {
    f3 o, p, au, d;
    f3 inv, invs;
    float tmax, mag_a;
    float omax;  // max |o_i| + |A|: bounds the segment-side coordinates (prefilter margin)
    int n0, n1, n2;
    bool has_inf;  // some 1/d_i is infinite (invs != inv)
};

__device__ __forceinline__ float sanitize_inv(float v) {
    return isinf(v) ? copysignf(FLT_MAX, v) : v;
}

__device__ __forceinline__ bool load_lane(int64_t s, int64_t nseg, const float *__restrict__ o,
                                          const float *__restrict__ p, const float *__restrict__ d,
                                          const float *__restrict__ tmax, Lane &L) {
    if (s >= nseg) {
        L.o = L.p = L.au = L.d = L.inv = L.invs = mk(0.f, 0.f, 0.f);
        L.tmax = 0.f;
        L.mag_a = 0.f;
        L.omax = 0.f;
        L.n0 = L.n1 = L.n2 = 0;
        L.has_inf = false;
        return false;
    }
    L.o = mk(o[3 * s], o[3 * s + 1], o[3 * s + 2]);
    L.p = mk(p[3 * s], p[3 * s + 1], p[3 * s + 2]);
    const f3 dd = mk(d[3 * s], d[3 * s + 1], d[3 * s + 2]);
    L.d = dd;
    L.tmax = tmax[s];
    // invDir(1 / ray.d.x, ...), dirIsNeg = invDir < 0  (photonbeambvh.cpp:690-691)
    L.inv = mk(1 / dd.x, 1 / dd.y, 1 / dd.z);
    L.invs = mk(sanitize_inv(L.inv.x), sanitize_inv(L.inv.y), sanitize_inv(L.inv.z));
    L.has_inf = isinf(L.inv.x) || isinf(L.inv.y) || isinf(L.inv.z);
    L.n0 = L.inv.x < 0;
    L.n1 = L.inv.y < 0;
    L.n2 = L.inv.z < 0;
    // A = a1 - a0; magA = |A|; A /= magA   (photonbeam.cpp:90-92, 121)
    const f3 A = sub3(L.p, L.o);
    L.mag_a = len3(A);
    L.au = (L.mag_a != 0.0f) ? div3(A, L.mag_a) : mk(0.f, 0.f, 0.f);
    L.omax = fmaxf(fmaxf(fabsf(L.o.x), fabsf(L.o.y)), fabsf(L.o.z)) + L.mag_a;
    return true;
}

// Conservative reject ahead of the exact closest-point code.  Every point the reference's
// ComputeClosestPoints returns lies (to within a few ulps of the largest coordinate involved) on the
// line a0 + s*au or b0 + t*bu, so its distance is at least the line-line distance
// |t.(au x bu)| / |au x bu| minus that rounding.  With |au x bu|^2 >= 1e-2 the beam-side parameter is
// bounded (|t1| <= |t|/|au x bu| <= 10|t|), so the coordinates, and the rounding, are bounded too;
// nearer-parallel pairs always take the exact path.  A pair rejected here cannot have a computed
// distance below R + r, so skipping it changes no result bit (the parity tests count every pair).
__device__ __forceinline__ bool far_from_lines(const Lane &L, const BeamV &r, float maxd) {
    if (L.mag_a == 0.0f) return false;
    const f3 t = sub3(r.b0, L.o);
    const f3 n = mk(L.au.y * r.bu.z - L.au.z * r.bu.y, L.au.z * r.bu.x - L.au.x * r.bu.z,
                    L.au.x * r.bu.y - L.au.y * r.bu.x);
    const float nn = lensq3(n);
    if (!(nn >= 1e-2f)) return false;
    const float tn = fabsf(dot3(t, n));
    const float tl = fabsf(t.x) + fabsf(t.y) + fabsf(t.z);
    const float bmax = fmaxf(fmaxf(fabsf(r.b0.x), fabsf(r.b0.y)), fabsf(r.b0.z));
    const float mag = L.omax + bmax + 10.0f * tl;       // bound on every coordinate involved
    const float eps = 1e-5f * mag + 1e-6f;               // >> the few-ulp rounding of those points
    const float nl = __builtin_sqrtf(nn);
    return (tn - 1e-6f * tl) > (maxd * 1.0001f + 2.0f * eps) * (nl + 1e-6f);
}

// far_from_lines with FMAs and the hardware sqrt: the same bound, evaluated to within a few ulps
// of the exact values, far inside its margins (1e-6 relative on |t.n|, |n| and the 1e-5 eps).
// Any rejection is still a proof that the reference's computed distance is >= maxd.
__device__ __forceinline__ bool far_from_lines_fast(f3 o, f3 au, float mag_a, float omax, f3 b0, f3 bu, float maxd) {
    if (mag_a == 0.0f) return false;
    const f3 t = sub3(b0, o);
    const f3 n = mk(__builtin_fmaf(au.y, bu.z, -(au.z * bu.y)), __builtin_fmaf(au.z, bu.x, -(au.x * bu.z)),
                    __builtin_fmaf(au.x, bu.y, -(au.y * bu.x)));
    const float nn = __builtin_fmaf(n.x, n.x, __builtin_fmaf(n.y, n.y, n.z * n.z));
    if (!(nn >= 1e-2f)) return false;
    const float tn = fabsf(__builtin_fmaf(t.x, n.x, __builtin_fmaf(t.y, n.y, t.z * n.z)));
    const float tl = fabsf(t.x) + fabsf(t.y) + fabsf(t.z);
    const float bmax = fmaxf(fmaxf(fabsf(b0.x), fabsf(b0.y)), fabsf(b0.z));
    const float mag = omax + bmax + 10.0f * tl;
    const float eps = 1e-5f * mag + 1e-6f;
    const float nl = __builtin_amdgcn_sqrtf(nn) * 1.000001f;  // v_sqrt_f32 (1 ulp) rounded up
    return (tn - 1e-6f * tl) > (maxd * 1.0001f + 2.0f * eps) * (nl + 1e-6f);
}

}  // namespace
}  // namespace bre
