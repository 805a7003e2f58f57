// bre_gather.hip — the beam-radiance gather on gfx950.
//
// One launch replaces the reference's per-segment loop body (photonbeam.cpp:494-508) for every
// camera segment of an iteration: PhotonBeamBVH::Intersect (photonbeambvh.cpp:685-723) becomes a
// traversal of the GPU BVH, and each beam reached is re-tested with the reference's own slab test
// on its own (group) box, so the candidate set is the reference's exactly; each candidate then
// runs ComputeClosestPoints and the 1D kernel 1e-5*powerEnd*sqrt(1-(d/(R+r))^2) in the
// reference's float arithmetic (bre_math.h).
//
// Kernels (BRE_OPT_KERNEL):
//   0 (default) / 4  k_gather_tile — the production gather.  A wave owns a packet of 64 segments
//                    (one per lane) and walks one BVH work root wave-uniformly down to LEAF TILES
//                    of up to 64 beams; per staged tile a packet-level bundle reject and a per-lane
//                    separable line-distance prefilter choose the (beam, lane) pairs that can
//                    contribute, and those run the reference's box test + ComputeClosestPoints +
//                    kernel 64 pairs at a time with every lane busy.  Kernel 0 builds the tile tree
//                    with BRE_OPT_TILE_LEAF beams per leaf, kernel 4 with BRE_OPT_LEAF_SIZE.
//   2                k_gather_thread — classic thread-per-segment traversal with a per-thread LDS
//                    stack: a structurally independent implementation kept as a cross-check.
//   5                the capsule-chunk index (bre_chunk.hip).
// Kernels 1, 3 and 6 of round 1 (depth-first wave packets, packet-proxy traversal and its
// hand-over mode) were slower than kernel 0 on every measured workload and are removed.
#include <hip/hip_runtime.h>

#include <float.h>

#include "bre_device.h"
#include "bre_lane.h"
#include "bre_math.h"

namespace bre {

namespace {

constexpr int kThreadBlock = 128;  // 2 waves, 32 KiB LDS stack

// The timing ablations of rounds 2-5 (BRE_ABLATE 2-5: no exact stage, no prefilter scan, traversal
// only, one racy accumulation round; BRE_NO_QCOUNT / BRE_NO_TAX) are not in the production source since
// round 6: profiles/r6/negative/ablation_switches_r6.patch restores them (and
// profiles/r5/negative/ablation_switches.patch the variants measured negative in rounds 2-4).  The two
// profiling builds below stay: profiles/phase_timing.py and profiles/scan_stats.py use them.
// BRE_PHASE_TIMING 1 (profiling builds only): the production tile kernel adds, per wave, the
// shader-clock cycles (s_memtime) of its phases into the counter block -- leaf staging into
// `candidates`, the prefilter scan into `contributions`, the exact stage into `node_visits`, the
// whole wave into `leaf_visits` (read back with the timing option); the reads serialise a little.
#ifndef BRE_PHASE_TIMING
#define BRE_PHASE_TIMING 0
#endif
// BRE_SQRT_NOSCALE 1 (default): the exact stage's two square roots without the compiler's small-input
// scaling (sqrt_cr_noscale, bit-identical results: see tile_exact); 0 = sqrtf
#ifndef BRE_SQRT_NOSCALE
#define BRE_SQRT_NOSCALE 1
#endif
// The exact stage reads the SegRec planes through a buffer descriptor (SGPR base + 32-bit lane offset:
// one VALU of address arithmetic instead of 64-bit pointer math; with the power too, C2 +0.8%, C3 +2%,
// profiles/r3b/run4).
// Raw buffer resource over [p, p + 4 GiB): offsets are 32-bit, out-of-range reads return 0.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void *p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, -1, 0x00020000);
}
__device__ __forceinline__ float4 buf_f4(__amdgpu_buffer_rsrc_t r, unsigned int voff, unsigned int soff) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, 0);
    return make_float4(__int_as_float(v[0]), __int_as_float(v[1]), __int_as_float(v[2]), __int_as_float(v[3]));
}
// BRE_SCAN_STATS 1 (profiling builds only): the production tile kernel adds, per wave, scan-shape
// sums into the counter block instead (profiles/scan_stats.py): lanes on the tile (candidates), kept
// beams (contributions), scan steps taken (node_visits), steps of a full (lane, beam) pair
// compaction ceil(on * kept / 64) (leaf_visits), leaf visits (beam_evals), queued pairs
// (useful_beam_evals), min(on, kept) (prefilter_rejects), transposed tiles (ccp_wave_evals)
#ifndef BRE_SCAN_STATS
#define BRE_SCAN_STATS 0
#endif
// BRE_WAVE_TIMES 1 (study builds only, profiles/r6/wave_times.py): every tile-kernel wave stores its
// start and end times (s_memrealtime, the device's 100 MHz clock) into a device array read back by
// bre_study_wave_times (exported by such builds only): the kernel's dispatch order and tail.
#ifndef BRE_WAVE_TIMES
#define BRE_WAVE_TIMES 0
#endif
#if BRE_WAVE_TIMES
constexpr int kWaveTimes = 1 << 22;
__device__ unsigned long long g_wave_t[2][kWaveTimes];
#endif
__device__ __forceinline__ void wave_time(int which, int lane) {
#if BRE_WAVE_TIMES
    if (lane == 0 && blockIdx.x < (unsigned)kWaveTimes) g_wave_t[which][blockIdx.x] = __builtin_amdgcn_s_memrealtime();
#else
    (void)which;
    (void)lane;
#endif
}
__device__ __forceinline__ unsigned long long phase_clock() {
    return BRE_PHASE_TIMING ? (unsigned long long)__builtin_amdgcn_s_memtime() : 0ull;
}

struct Prof {
    unsigned long long leaves = 0, beams = 0, ccp_waves = 0, rejects = 0, useful = 0, queued = 0;
};

__device__ __forceinline__ int lanes_below(unsigned long long m) {
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

// ---------------------------------------------------------------------------------------------
// Kernel 2 helpers: evaluate one beam record for one lane — reference box test, closest points,
// kernel (photonbeam.cpp:495-507) — and write the lane's results.
template <bool COUNT>
__device__ __forceinline__ void eval_beam(const Lane &L, bool lane_on, const BeamV &r, const float4 *__restrict__ pw,
                                          int64_t bi, float R, float &cr, float &cg, float &cb, int &cand,
                                          int &contrib) {
    // candidate: the reference's own slab test on the beam's (group) box.  For a lane whose 1/d has
    // no infinite component, node_test(box, inv) is the same decision (bre_math.h); lanes with an
    // axis-parallel direction (inf, possible NaN paths) take the literal statement.
    float te;
    bool hit = lane_on & node_test(r.box, L.o, L.invs, L.tmax, te);
    if (L.has_inf) hit = lane_on & slab_test(r.box, L.o, L.inv, L.n0, L.n1, L.n2, L.tmax, nullptr);
    if (COUNT) cand += hit;
    if (!hit) return;
    const float maxd = R + r.radius;  // MaxDistance = currentBeamRadius + beam->radius
    float dist;
    const bool ok = closest_distance(L.o, L.p, L.au, L.mag_a, r.b0, r.bu, r.mag_b, dist);
    if (ok & (dist < maxd)) {
        const float rr = dist / maxd;
        const float w = sqrtf(1.0f - rr * rr);
        const float4 pv = pw[bi];
        cr += pv.x * w;
        cg += pv.y * w;
        cb += pv.z * w;
        ++contrib;
    }
}

template <bool COUNT>
__device__ __forceinline__ void finish_lane(int64_t s, bool valid, float cr, float cg, float cb, int cand, int contrib,
                                            unsigned long long visits, const int32_t *__restrict__ pixel, int64_t npix,
                                            float *__restrict__ accum, float *__restrict__ seg_rgb,
                                            int32_t *__restrict__ seg_counts, DevCounters *ctr) {
    if (valid) {
        if (seg_rgb) {
            seg_rgb[3 * s] = cr;
            seg_rgb[3 * s + 1] = cg;
            seg_rgb[3 * s + 2] = cb;
        }
        if (accum) {
            const int32_t px = pixel[s];
            if (px < 0 || px >= npix) {
                atomicOr(&ctr->flags, kFlagPixel);
            } else if (cr != 0.f || cg != 0.f || cb != 0.f) {
                atomicAdd(&accum[3 * (int64_t)px], cr);
                atomicAdd(&accum[3 * (int64_t)px + 1], cg);
                atomicAdd(&accum[3 * (int64_t)px + 2], cb);
            }
        }
        if (seg_counts) {
            seg_counts[2 * s] = COUNT ? cand : -1;
            seg_counts[2 * s + 1] = contrib;
        }
    }
    if (COUNT) {
        unsigned long long c = valid ? (unsigned long long)cand : 0ull;
        unsigned long long k = valid ? (unsigned long long)contrib : 0ull;
        unsigned long long v = visits;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            c += __shfl_xor(c, off);
            k += __shfl_xor(k, off);
            v += __shfl_xor(v, off);
        }
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(&ctr->candidates, c);
            atomicAdd(&ctr->contributions, k);
            atomicAdd(&ctr->node_visits, v);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Packet bundle for the packet-level line-distance reject.  A line C (point co, unit direction cu)
// and delta >= the distance of every valid lane's segment END POINTS from C.  The distance to a line
// is convex along a segment, so every point of every lane's segment lies within delta of C, and for
// any beam line B: dist(segment_i, B) >= dist(C, B) - delta.  One lane-wide evaluation per beam (64
// beams at once) then rejects a beam for all 64 segments, before the per-lane prefilter.  delta and
// the coordinate bound are inflated for rounding.
struct Bundle {
    f3 co, cu;
    float delta;  // FLT_MAX disables the test
    float omax;   // max over valid lanes of Lane::omax (bounds every segment-side coordinate)
    // packet capsule of the lanes' RAYS [o, o + tmax d] (what the reference's box test sees): every
    // ray point is co + s cu + w with s in [s0, s1] and |w| <= gbox (rounding margins included);
    // gbox = FLT_MAX disables the box reject
    float s0, s1, gbox;
    f3 icu;       // 1 / cu with infinities replaced by +-FLT_MAX
    f3 q;         // co x cu (the separable line reject, bundle_far_sep)
    float col1;   // |co|_1
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
    return v;
}
__device__ __forceinline__ float readlane_f(float v, int i) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), i)); }
__device__ __forceinline__ float uniform_f(float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); }

// The whole packet's bundle, wave-uniform (kept in SGPRs).  All lanes must call.
__device__ __forceinline__ Bundle make_bundle(const Lane &L, bool valid) {
    const int cnt = __popcll(__ballot(valid));
    const float n = (float)(cnt > 0 ? cnt : 1);
    Bundle K;
    K.co = mk(wave_sum(valid ? L.o.x : 0.f) / n, wave_sum(valid ? L.o.y : 0.f) / n, wave_sum(valid ? L.o.z : 0.f) / n);
    const f3 su = mk(wave_sum(valid ? L.au.x : 0.f), wave_sum(valid ? L.au.y : 0.f), wave_sum(valid ? L.au.z : 0.f));
    const float sl = sqrtf(lensq3(su));
    K.omax = wave_max(valid ? L.omax : 0.f);
    bool ok = cnt > 0 && sl > 0.f && isfinite(sl);
    K.cu = ok ? mk(su.x / sl, su.y / sl, su.z / sl) : mk(0.f, 0.f, 1.f);
    {
        // the line through the centres of the origins' and the end points' boxes: closer to the
        // minimax line than the mean line when the lanes' lengths differ (any line is valid: delta is
        // measured from it)
        const auto ctr = [&](float v) {
            const float hi = wave_max(valid ? v : -FLT_MAX), lo = -wave_max(valid ? -v : -FLT_MAX);
            return 0.5f * lo + 0.5f * hi;
        };
        const f3 a = mk(ctr(L.o.x), ctr(L.o.y), ctr(L.o.z)), b = mk(ctr(L.p.x), ctr(L.p.y), ctr(L.p.z));
        const f3 ab = sub3(b, a);
        const float l = sqrtf(lensq3(ab));
        if (cnt > 0 && l > 1e-6f * (1.f + fabsf(a.x) + fabsf(a.y) + fabsf(a.z)) && isfinite(l) && isfinite(a.x) &&
            isfinite(a.y) && isfinite(a.z)) {
            K.co = a;
            K.cu = mk(ab.x / l, ab.y / l, ab.z / l);
            ok = true;
        }
    }
    const auto perp = [&](f3 x) {
        const f3 t = sub3(x, K.co);
        const f3 c = mk(t.y * K.cu.z - t.z * K.cu.y, t.z * K.cu.x - t.x * K.cu.z, t.x * K.cu.y - t.y * K.cu.x);
        return sqrtf(lensq3(c));
    };
    const float dl = valid ? fmaxf(perp(L.o), perp(L.p)) : 0.f;
    const float cm = fmaxf(fmaxf(fabsf(K.co.x), fabsf(K.co.y)), fabsf(K.co.z));
    const float d = wave_max(dl);
    K.delta = (ok && isfinite(d)) ? d * 1.0001f + 1e-5f * (K.omax + cm) + 1e-6f : FLT_MAX;
    // the rays' capsule around C for the box reject (bundle_box_miss)
    {
        const f3 q = add3(L.o, scale3(L.d, L.tmax));  // far end of the reference's ray extent
        const float qm = fmaxf(fmaxf(fabsf(q.x), fabsf(q.y)), fabsf(q.z));
        const bool fin = !valid || (isfinite(qm) && isfinite(L.omax));
        const float so = dot3(sub3(L.o, K.co), K.cu), sq = dot3(sub3(q, K.co), K.cu);
        const float db = valid ? fmaxf(perp(L.o), perp(q)) : 0.f;
        const float dmax = wave_max(db);
        const float smax = wave_max(valid ? fmaxf(so, sq) : -FLT_MAX);
        const float smin = -wave_max(valid ? -fminf(so, sq) : -FLT_MAX);
        const float mb = fmaxf(K.omax, wave_max(valid ? qm : 0.f)) + cm;
        const bool all_fin = __ballot(!fin) == 0ull;
        const float mg = 1e-5f * mb + 1e-6f;
        K.gbox = (ok && all_fin && isfinite(dmax) && isfinite(mb)) ? dmax * 1.0001f + mg : FLT_MAX;
        K.s0 = smin - mg;
        K.s1 = smax + mg;
        K.icu = mk(sanitize_inv(1.0f / K.cu.x), sanitize_inv(1.0f / K.cu.y), sanitize_inv(1.0f / K.cu.z));
    }
    K.co = mk(uniform_f(K.co.x), uniform_f(K.co.y), uniform_f(K.co.z));
    K.cu = mk(uniform_f(K.cu.x), uniform_f(K.cu.y), uniform_f(K.cu.z));
    K.delta = uniform_f(K.delta);
    K.omax = uniform_f(K.omax);
    K.gbox = uniform_f(K.gbox);
    K.s0 = uniform_f(K.s0);
    K.s1 = uniform_f(K.s1);
    K.icu = mk(uniform_f(K.icu.x), uniform_f(K.icu.y), uniform_f(K.icu.z));
    K.q = mk(K.co.y * K.cu.z - K.co.z * K.cu.y, K.co.z * K.cu.x - K.co.x * K.cu.z, K.co.x * K.cu.y - K.co.y * K.cu.x);
    K.col1 = fabsf(K.co.x) + fabsf(K.co.y) + fabsf(K.co.z);
    return K;
}

// Packet-level box reject.  A pair is a candidate only if the lane's ray hits the beam's (group) box
// (the reference's slab test, photonbeambvh.cpp:685-723); every lane's ray lies in the capsule
// {co + s cu + w : s in [s0, s1], |w| <= gbox}, which meets the box only if the piece C[s0, s1]
// crosses the box grown by gbox.  If it does not, no lane can hit the box (gbox and the s-range carry
// 1e-5 of the coordinate bound: far above the reference test's own rounding and its gamma(3)
// far-plane pad), so the beam is no lane's candidate and is skipped for the whole packet.
// A box with a NaN coordinate is never rejected here.
__device__ __forceinline__ bool bundle_box_miss(const Bundle &K, const Box6 &b) {
    if (!(K.gbox < 1e30f)) return false;
    // A plane within ~gbox of the capsule has |coordinate| <= ~2 x the packet's coordinate bound, so
    // the packet-side margin already covers its rounding; farther planes cannot flip the decision.
    const float bsum = (b.lx + b.ly) + (b.lz + b.hx) + (b.hy + b.hz);
    const float g = K.gbox;
    const float ax = (b.lx - g - K.co.x) * K.icu.x, cx = (b.hx + g - K.co.x) * K.icu.x;
    const float ay = (b.ly - g - K.co.y) * K.icu.y, cy = (b.hy + g - K.co.y) * K.icu.y;
    const float az = (b.lz - g - K.co.z) * K.icu.z, cz = (b.hz + g - K.co.z) * K.icu.z;
    const float tn = fmaxf(fmaxf(fminf(ax, cx), fminf(ay, cy)), fmaxf(fminf(az, cz), K.s0));
    const float tf = fminf(fminf(fmaxf(ax, cx), fmaxf(ay, cy)), fminf(fmaxf(az, cz), K.s1));
    return (bsum == bsum) & (tn > tf);
}

// Packet-level line reject of a beam: a rejection proves that every lane's computed
// ComputeClosestPoints distance is >= maxd.  Every lane's segment lies within delta of the bundle
// line C, so its distance from the beam LINE B is >= D(C, B) - delta.  The reference's pA lies on
// the segment to within 10U Ma + U Ol (U = 2^-24; see the margin note above ScanLane), and its pB on
// line B to within 2U |t1| + U Bl; a pair can only contribute if |pA - pB| < maxd, which puts pB
// within maxd of pA, so |t1| <= |pB - b0| <= Ol + Ma + maxd + Bl: pB is within 2U (Ol + Ma + maxd + Bl)
// + U Bl of the line, whatever the pair's angle.  So |pA - pB| >= D(C, B) - delta - eps with
// eps = U (12 Ma + 3 Ol + 3 Bl + 2 maxd) <= U (21 omax + 3 Bl + 2 maxd) (omax bounds max|o_i| + Ma
// over the lanes, Ol <= 3 max|o_i|), and the reference's rounded distance is >= maxd whenever
// D(C, B) > maxd (1 + 5U) + delta + eps.  D(C, B) = |t.n| / |n| is evaluated with fmas (error
// <= 8U |t|_1, absorbed by the 1e-6 |t|_1 slack; |n| rounded up), only for |n|^2 >= 1e-2.  Margin
// mode 1 uses twice eps: 2.5e-6 omax + 3.6e-7 Bl + 2.4e-7 maxd + 1e-6; mode 0 keeps round 2's
// 2e-5 (omax + bmax + 10 |t|_1 + maxd + 1) + 2e-6 and the 1e-4 relative factor.
__device__ __forceinline__ bool bundle_far(const Bundle &K, f3 b0, f3 bu, float maxd, int margin) {
    if (!(K.delta < 1e30f)) return false;
    const f3 t = sub3(b0, K.co);
    const f3 n = mk(__builtin_fmaf(K.cu.y, bu.z, -(K.cu.z * bu.y)), __builtin_fmaf(K.cu.z, bu.x, -(K.cu.x * bu.z)),
                    __builtin_fmaf(K.cu.x, bu.y, -(K.cu.y * bu.x)));
    const float nn = __builtin_fmaf(n.x, n.x, __builtin_fmaf(n.y, n.y, n.z * n.z));
    if (!(nn >= 1e-2f)) return false;
    const float tn = fabsf(__builtin_fmaf(t.x, n.x, __builtin_fmaf(t.y, n.y, t.z * n.z)));
    const float tl = fabsf(t.x) + fabsf(t.y) + fabsf(t.z);
    float lim;
    if (margin) {
        const float b1 = fabsf(b0.x) + fabsf(b0.y) + fabsf(b0.z);
        lim = (maxd + K.delta) * 1.000001f + (2.5e-6f * K.omax + 3.6e-7f * b1 + 2.4e-7f * maxd + 1e-6f);
    } else {
        const float bmax = fmaxf(fmaxf(fabsf(b0.x), fabsf(b0.y)), fabsf(b0.z));
        const float mag = K.omax + bmax + 10.0f * tl + maxd + 1.0f;
        lim = (maxd + K.delta) * 1.0001f + 2.0f * (1e-5f * mag + 1e-6f);
    }
    const float nl = __builtin_amdgcn_sqrtf(nn) * 1.000001f;
    return (tn - 1e-6f * tl) > lim * (nl + 1e-6f);
}

// The same packet-level line reject in the scan's separable form (margin mode 1): the bundle line
// C = (co, cu) plays a lane whose margin is delta, so t.n = cu.m0 - bu.(co x cu) reuses the beam's
// staged m0 = bu x b0 and |n|^2 is bracketed by c = cu.bu, no cross product or square root per beam.
// The computed t.n is within 14U (Bl + |co|_1) of the exact one (the ScanLane analysis with o -> co,
// au -> cu), i.e. D(C, B) within 140.1U (Bl + |co|_1) for |n| > 0.0999 (u >= 0.0101); with eps above,
// rejecting D(C, B) > thr_b = (maxd + delta) 1.000001 + 1.93e-5 (Bl + |co|_1) + 2.5e-6 omax + 2.4e-7 Mb
// + 1e-6 (twice both terms) proves every lane's reference distance >= maxd.  delta = FLT_MAX (the
// reject disabled) squares to +inf: never a reject.
__device__ __forceinline__ bool bundle_far_sep(const Bundle &K, f3 b0, f3 bu, f3 m0, float maxd, float mag_b) {
    const float c = __builtin_fmaf(K.cu.x, bu.x, __builtin_fmaf(K.cu.y, bu.y, K.cu.z * bu.z));
    const float u = __builtin_fmaf(-c, c, 1.0001f);
    const float x = __builtin_fmaf(K.cu.x, m0.x, __builtin_fmaf(K.cu.y, m0.y, K.cu.z * m0.z));
    const float t = __builtin_fmaf(-bu.x, K.q.x, __builtin_fmaf(-bu.y, K.q.y, __builtin_fmaf(-bu.z, K.q.z, x)));
    const float b1 = fabsf(b0.x) + fabsf(b0.y) + fabsf(b0.z);
    const float thr = (maxd + K.delta) * 1.000001f + 1.93e-5f * (b1 + K.col1) + 2.5e-6f * K.omax + 2.4e-7f * mag_b + 1e-6f;
    return (u >= 0.0101f) & ((t * t) > (thr * thr) * u);
}

// ---------------------------------------------------------------------------------------------
// Per-lane tile line reject (option 112 = 1).  A contributing pair (lane i, beam j) has the reference's
// pA on segment i (to rounding) and pB on beam j's line with |pA - pB| < maxd_j, so pB lies in the box
// of the launch's segments grown by maxd_j.  k_tile_axis gives every tile an axis line such that every
// beam LINE of the tile, clipped to that box (plus a margin), lies within rho of it (distance to a line
// is convex along a line, so the clipped piece's two end points bound it).  Then
//   D(line_i, axis) <= d(pA, axis) <= |pA - pB| + d(pB, axis) < maxd_j + rho,
// so a lane whose segment LINE is farther than rho + maxd_max from the axis line has no pair in the
// tile that can contribute.  The test is the scan's own separable line-distance test
// (scan_keep_mask) with the axis as a pseudo-beam whose threshold is rho + Ab' (Ab' with the tile's
// largest |b0|_1 and |B|, so the scan's rounding analysis covers every beam of the tile): per leaf
// visit one 14-VALU test per lane, before the tile is staged.  Lanes it rejects are taken off the tile
// (fewer lanes on: more tiles take the transposed scan), and a tile no lane keeps is not staged at all.
// Only the production instantiation tests (the counting one box-tests every beam of a visited tile for
// C); the rejected pairs never contribute, so the queues differ only by non-contributing pairs and
// every per-segment sum is bit-identical (tests/test_prefilter_options_gpu.py).
__device__ __forceinline__ unsigned int ord_u(float f) {
    const unsigned int u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord_f(unsigned int u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

__global__ void k_segbox_init(unsigned int *__restrict__ b) {
    if (threadIdx.x < 6) b[threadIdx.x] = threadIdx.x < 3 ? 0xffffffffu : 0u;
}

// box of the launch's finite segment end points (6 ordered uints: min xyz, max xyz).  Grid-stride
// over a bounded grid, reduced per wave and then per block in LDS: one set of six atomics per block
// (per-wave atomics on the same six words serialised at the L2: 0.64 ms at C2's 0.6M segments)
constexpr int kSegboxBlocks = 512;
// the kernels around the gather run in one-wave workgroups (bre_slot.hip: they then fit the slots a
// concurrent gather's retiring waves free, so the pipelined pass chain runs inside the other gather)
constexpr int kPassBlock = 64;
__global__ __launch_bounds__(kPassBlock) void k_segbox(int64_t nseg, const float *__restrict__ o, const float *__restrict__ p,
                                                unsigned int *__restrict__ b) {
    __shared__ unsigned int red[kPassBlock / 64][6];
    unsigned int mn[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, mx[3] = {0u, 0u, 0u};
    for (int64_t i = (int64_t)blockIdx.x * kPassBlock + threadIdx.x; i < nseg; i += (int64_t)gridDim.x * kPassBlock) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const float *q = (e ? p : o) + 3 * i;
            const float v[3] = {q[0], q[1], q[2]};
            if (isfinite(v[0]) && isfinite(v[1]) && isfinite(v[2])) {
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    mn[k] = min(mn[k], ord_u(v[k]));
                    mx[k] = max(mx[k], ord_u(v[k]));
                }
            }
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            mn[k] = min(mn[k], (unsigned int)__shfl_xor((int)mn[k], off));
            mx[k] = max(mx[k], (unsigned int)__shfl_xor((int)mx[k], off));
        }
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            red[w][k] = mn[k];
            red[w][3 + k] = mx[k];
        }
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int k = threadIdx.x;
        unsigned int v = red[0][k];
        for (int j = 1; j < kPassBlock / 64; ++j) v = k < 3 ? min(v, red[j][k]) : max(v, red[j][k]);
        if (k < 3)
            atomicMin(&b[k], v);
        else
            atomicMax(&b[k], v);
    }
}

// One wave per leaf tile: axis = mean start -> mean end of its usable beams, rho = the largest
// distance of a clipped beam line's end points from the axis (with rounding margins), stored as the
// pseudo-beam record the per-lane tile line reject tests (TileAxis).
__global__ __launch_bounds__(64) void k_tile_axis(const BeamRec *__restrict__ recs, BeamSet bset, int64_t nvalid,
                                                  int leaf_size,
                                                  const unsigned int *__restrict__ segb, float R,
                                                  TileAxis *__restrict__ out) {
    const int64_t tile = blockIdx.x;
    const int lane = threadIdx.x;
    const int64_t j = tile * leaf_size + lane;
    bool ok = lane < leaf_size && j < nvalid;
    f3 b0 = mk(0.f, 0.f, 0.f), bu = mk(0.f, 0.f, 0.f);
    float mb = 0.f, rad = 0.f;
    if (ok) {
        const BeamV r = load_beam(recs, j, bset);
        b0 = r.b0;
        bu = r.bu;
        mb = r.mag_b;
        rad = r.radius;
        // a zero-length or non-finite beam has a NaN / infinite reference box: never a candidate
        ok = mb > 0.f && isfinite(mb) && isfinite(b0.x) && isfinite(b0.y) && isfinite(b0.z) && isfinite(bu.x) &&
             isfinite(bu.y) && isfinite(bu.z) && isfinite(rad);
    }
    const float rmax = wave_max(ok ? rad : 0.f);
    const float n = wave_sum(ok ? 1.f : 0.f);
    TileAxis A;
    if (n == 0.f || !(segb[0] <= segb[3] && segb[1] <= segb[4] && segb[2] <= segb[5])) {
        // no usable beam (or no finite segment): nothing of this tile can contribute
        A.d[0] = 1.f;
        A.d[1] = A.d[2] = 0.f;
        A.thr = 0.f;
        A.m[0] = A.m[1] = A.m[2] = 0.f;
        A.grow = -1.f;
        if (lane == 0) out[tile] = A;
        return;
    }
    const f3 e = add3(b0, scale3(bu, mb));
    // the axis through the centres of the starts' and the ends' boxes (round 5: C2 +1.2% over the
    // mean start -> mean end, profiles/r5/run3)
    const auto ctr = [&](float v) {
        const float hi = wave_max(ok ? v : -FLT_MAX), lo = -wave_max(ok ? -v : -FLT_MAX);
        return 0.5f * lo + 0.5f * hi;
    };
    const f3 ps = mk(ctr(b0.x), ctr(b0.y), ctr(b0.z));
    const f3 pe = mk(ctr(e.x), ctr(e.y), ctr(e.z));
    f3 d = sub3(pe, ps);
    const float dl = sqrtf(lensq3(d));
    d = (dl > 1e-6f * (1.f + fabsf(ps.x) + fabsf(ps.y) + fabsf(ps.z)) && isfinite(dl)) ? scale3(d, 1.f / dl)
                                                                                      : mk(1.f, 0.f, 0.f);
    // the region: segment box grown by maxd_max = R + rmax, plus margins
    const float lo[3] = {ord_f(segb[0]), ord_f(segb[1]), ord_f(segb[2])};
    const float hi[3] = {ord_f(segb[3]), ord_f(segb[4]), ord_f(segb[5])};
    const float cm = fmaxf(fmaxf(fmaxf(fabsf(lo[0]), fabsf(lo[1])), fmaxf(fabsf(lo[2]), fabsf(hi[0]))),
                           fmaxf(fabsf(hi[1]), fabsf(hi[2])));
    const float grow = (R + rmax) * 1.001f + 1e-5f * cm + 1e-6f;
    float dist = 0.f;
    if (ok) {
        const float o3[3] = {b0.x, b0.y, b0.z}, u3[3] = {bu.x, bu.y, bu.z};
        float t0 = -FLT_MAX, t1 = FLT_MAX;
        bool in = true;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float l = lo[k] - grow, h = hi[k] + grow;
            if (u3[k] == 0.f) {
                in = in && o3[k] >= l && o3[k] <= h;
            } else {
                float a = (l - o3[k]) / u3[k], c = (h - o3[k]) / u3[k];
                if (a > c) {
                    const float x = a;
                    a = c;
                    c = x;
                }
                t0 = fmaxf(t0, a);
                t1 = fminf(t1, c);
            }
        }
        if (in && t0 <= t1) {
            // widen the piece by a little (the slab parameters carry rounding)
            const float tw = 1e-5f * (fabsf(t0) + fabsf(t1)) + 1e-6f;
            t0 -= tw;
            t1 += tw;
            const auto dax = [&](float t) {
                const f3 q = sub3(add3(b0, scale3(bu, t)), ps);
                const f3 c = mk(q.y * d.z - q.z * d.y, q.z * d.x - q.x * d.z, q.x * d.y - q.y * d.x);
                return sqrtf(lensq3(c));
            };
            dist = fmaxf(dax(t0), dax(t1));
            // a NaN distance must not shrink rho: treat it as unbounded
            if (!(dist == dist)) dist = FLT_MAX;
        }
    }
    const float rho_raw = wave_max(dist);
    const float pm = fmaxf(fmaxf(fabsf(ps.x), fabsf(ps.y)), fabsf(ps.z));
    const float rho = rho_raw * 1.0001f + 1e-5f * (cm + pm + grow) + 1e-6f;
    // the scan's beam-side margin Ab' (make_scan_beam) with maxd_max and the tile's largest |b0|_1 and
    // |B| (the separable form evaluates t.n at the axis point: its |p|_1 joins the max)
    const float b1 = wave_max(ok ? fabsf(b0.x) + fabsf(b0.y) + fabsf(b0.z) : 0.f);
    const float p1 = fabsf(ps.x) + fabsf(ps.y) + fabsf(ps.z);
    const float bmag = wave_max(ok ? mb : 0.f);
    const float ab = (R + rmax) * 1.000001f + 1.93e-5f * fmaxf(b1, p1) + 2.4e-7f * bmag + 1e-6f;
    const float thr = (rho + ab) * 1.0001f + 1e-6f;
    A.d[0] = d.x;
    A.d[1] = d.y;
    A.d[2] = d.z;
    A.thr = (rho_raw < FLT_MAX && isfinite(thr)) ? thr : FLT_MAX;  // FLT_MAX: never a reject
    A.m[0] = d.y * ps.z - d.z * ps.y;  // m = d x p (the scan's m0 = bu x b0)
    A.m[1] = d.z * ps.x - d.x * ps.z;
    A.m[2] = d.x * ps.y - d.y * ps.x;
    A.grow = grow;
    if (lane == 0) out[tile] = A;
}

// ---------------------------------------------------------------------------------------------
// Kernel 0/4 (k_gather_tile): wave-packet traversal over leaf TILES of up to 64 beams.
//
// At dense candidate sets (the C2 Cornell fog: a camera segment passes ~16% of all beam boxes,
// and packets of incoherent bounce segments share few of them) the exact per-pair code executed
// under a 64-lane mask is the cost: a wave would run ComputeClosestPoints whenever ANY lane needs
// it, with a few % of the lanes active.  Per visited leaf tile:
//   1. lane j loads beam j of the tile and keeps its scan values in REGISTERS (7 VGPRs);
//   2. the packet bundle test (one beam per lane) drops beams far from every segment of the packet;
//   3. each lane runs the separable line-distance prefilter on the kept beams, the beam's values
//      broadcast from their lane by v_readlane into SGPRs; (beam, lane) pairs that pass are
//      appended to a per-wave LDS ring, one 32-bit entry each (ballot + mbcnt);
//   4. every 64 queued pairs run, one pair per lane with all lanes busy, the reference's box test
//      on the beam's (group) box, ComputeClosestPoints and the kernel, with the segment read back
//      from its 64-B record (k_seg_prep) through the vector cache, and add the contribution to the
//      segment's LDS accumulator.
// r2 profile of the round-1 form (tile staged in LDS, segment fields moved by 14 ds_bpermutes per
// batch): LDS array busy 60% of the kernel's clocks and 52% of the wave cycles stalled on LDS issue,
// VALU issue 22%; this form moves ~2.5x fewer LDS instructions.
// The prefilters only drop pairs with a computed distance >= R + r, which never contribute, and the
// box test is the reference's own, so the contributing pairs and each pair's value are the
// reference's; a segment's pairs are summed in queue order (leaf, beam, lane), fixed by the
// traversal: deterministic.
//
// Separable prefilter.  With t = b0 - o and n = au x bu,
//   t.n = au.(bu x b0) - bu.(o x au) = au.m0 - bu.q,
// so per (lane, beam) only two dot products and c = au.bu remain: m0 is held per beam, q per lane.
// |n|^2 = |au|^2|bu|^2 - c^2 (Lagrange) is bracketed by 0.99999 - c^2 <= |n|^2 <= 1.00001 - c^2
// (unit vectors to ~1e-7, c to ~5e-7).  A pair is rejected only when |n|^2 >= 1e-2 (|n| > 0.0999)
// and |t.n| > thr |n| with thr = Ab' + Al' (scan_need evaluates this without a square root).
//
// Margins (margin mode 1, the default since round 3).  U = 2^-24; L1 norms Ol = |o|_1, Bl = |b0|_1;
// Ma = |A|, Mb = |B|.  D = |t.n| / |n| is the exact distance of the lines o + s au and b0 + s bu (the
// stored float vectors, exact arithmetic).  Every point ComputeClosestPoints (photonbeam.cpp:87-186)
// returns lies near one of those lines:
//   * pA = a0 + au t0 with t0 in [0, Ma], or a0 + au d with d in [0, Ma]: the float products and sums
//     move it at most 2U Ma + U Ol off the line; pA = a0 is on it; pA = a1 is within 10U Ma of it
//     (au is (a1 - a0) rounded, scaled by the rounded 1 / |A|: a few U of direction);
//   * pB = b0 + bu d with d in [0, Mb]: within 2U Mb + U Bl; pB = b0 + bu t1 (the quirk of :178-181,
//     t1 outside [0, Mb]): within 2U |t1| + U Bl, and with |n| > 0.0999 the closest-point parameter
//     is |t1| <= |t| / |n| <= 10.1 (Bl + Ol) (the float Cramer solution adds ~100U |t|), so
//     within 20.2U (Bl + Ol) + U Bl.
// So |pA - pB| >= D - eps, eps = U (21.2 (Bl + Ol) + 10 Ma + 2 Mb), and the reference's float
// distance (difference, three squares, sum, correctly rounded sqrt) is >= (D - eps)(1 - 4U): it is
// >= maxd whenever D >= maxd (1 + 5U) + eps.  The scan's t.n = x - bu.q (m0 = bu x b0 and q = o x au
// rounded, two 3-term fma dot products) is within Et = 14U (Bl + Ol) of the exact t.n, so a reject
// (|t.n|_computed > thr |n|) gives D > thr - Et / |n| >= thr - 140.1U (Bl + Ol).  Hence
//   thr >= maxd (1 + 5U) + U (161.3 (Bl + Ol) + 10 Ma + 2 Mb)
// proves that every reference-computed distance of a rejected pair is >= maxd.  The kernel uses
// twice the U terms: Ab' = maxd * 1.000001 + 1.93e-5 Bl + 2.4e-7 Mb + 1e-6 (the absolute 1e-6 keeps
// thr clear of underflow), Al' = 1.93e-5 Ol + 1.2e-6 Ma.  For a unit-box scene that is ~6e-5 over
// maxd -- margin mode 0 (the round-2 bound, 2e-5 (omax + 10 |o|_1) + 1e-4 omax on each side) added
// ~1.4e-3, which at the late C2 iterations (maxd ~ 3e-3) queued ~1.4x the contributing pairs.
// Near-parallel pairs (|n|^2 possibly < 1e-2) and zero-length segments (Al' = FLT_MAX) are never
// rejected.  tests/test_margin_bound.py checks the bound against the oracle's ComputeClosestPoints on
// pairs placed just outside the threshold.
struct ScanLane {
    f3 q;       // o x au
    float al;   // Al' (see above);  FLT_MAX for a zero-length segment
};

__device__ __forceinline__ ScanLane make_scan_lane(const Lane &L, int margin) {
    ScanLane S;
    S.q = mk(L.o.y * L.au.z - L.o.z * L.au.y, L.o.z * L.au.x - L.o.x * L.au.z, L.o.x * L.au.y - L.o.y * L.au.x);
    const float o1 = fabsf(L.o.x) + fabsf(L.o.y) + fabsf(L.o.z);
    const float al = margin ? 1.93e-5f * o1 + 1.2e-6f * L.mag_a : 2e-5f * (L.omax + 10.0f * o1) + 1e-4f * L.omax;
    S.al = L.mag_a == 0.0f ? FLT_MAX : al;
    return S;
}

// The beam side of the scan: bu, m0 = bu x b0 and Ab' (maxd = R + r folded in).
struct ScanBeam {
    f3 bu, m0;
    float ab;
};

__device__ __forceinline__ ScanBeam make_scan_beam(const BeamV &r, float R, int margin) {
    const float maxd = R + r.radius;
    ScanBeam B;
    B.bu = r.bu;
    B.m0 = mk(r.bu.y * r.b0.z - r.bu.z * r.b0.y, r.bu.z * r.b0.x - r.bu.x * r.b0.z, r.bu.x * r.b0.y - r.bu.y * r.b0.x);
    const float b1 = fabsf(r.b0.x) + fabsf(r.b0.y) + fabsf(r.b0.z);
    if (margin) {
        B.ab = maxd * 1.000001f + 1.93e-5f * b1 + 2.4e-7f * r.mag_b + 1e-6f;
    } else {
        const float bmax = fmaxf(fmaxf(fabsf(r.b0.x), fabsf(r.b0.y)), fabsf(r.b0.z));
        // Ab = maxd 1.0001 + 2e-5 (bmax + 10 |b0|_1) + 2e-6, Eb = 1e-5 bmax + 1e-6
        B.ab = maxd * 1.0001f + 2e-5f * (bmax + 10.0f * b1) + 2e-6f + 10.0f * (1e-5f * bmax + 1e-6f);
    }
    return B;
}

// Beam j's scan values from the tile staged in LDS (two broadcast ds_read_b128): (bu, thr_sq) and
// (m0, 1.0001).  The stored constant is the u' constant of scan_need, so every loaded component has
// a use (a read whose w is unused is narrowed to ds_read_b96: 8 LDS cycles per wave, not 4).
struct ScanStaged {
    f3 bu, m0;
    float thr_sq;  // fl(thr * |thr|), thr = Ab' + the packet's max Al'; -inf: rejected; +inf: never
    float uc;      // 1.0001
};
__device__ __forceinline__ ScanStaged scan_beam_lds(const float4 (*tile)[2], int j) {
    const float4 a = tile[j][0], b = tile[j][1];
    ScanStaged B;
    B.bu = mk(a.x, a.y, a.z);
    B.thr_sq = a.w;
    B.m0 = mk(b.x, b.y, b.z);
    B.uc = b.w;
    return B;
}

// The per-(lane, beam) prefilter.  The pair is rejected iff
//   |n|^2 >= ~1e-2  and  tn > thr * |n|          (the separable bound above)
// and `need` is the complement.  Squares, no square root of |n|:
//   reject  <=>  u >= 0.0101  and  fl(tn * tn) > fl(thr_sq * u),   u = fl(1.0001 - c^2).
// thr is per BEAM: Ab' plus the largest Al' of the packet's lanes (>= each lane's own Al', so the
// bound above still proves every reject), and thr_sq = fl(thr * |thr|) is staged with the tile.
// For thr > 0 this implies tn > thr * |n| for the exact cross product n of the stored unit vectors:
// by the bracket above |n|^2 <= 1.00001 - c^2, and u >= (1.0001 - c^2)(1 - 2^-24) >= |n|^2 + 8.9e-5;
// the three roundings are at most 3 * 2^-24 relative, so tn^2 > thr^2 u (1 - 1.8e-7) > thr^2 |n|^2.
// u >= 0.0101 means c^2 <= 0.99 (to rounding), so |n|^2 >= 0.99999 - c^2 > 0.00999 (bracket):
// |n| > 0.0999, as the margin bound requires.  No underflow can fake a reject: thr >= Ab' > 1e-6 and
// u >= 0.0101 keep the right side >= 1e-14; an overflowing tn^2 really exceeds a finite right side;
// NaN compares keep the pair.  thr_sq = +inf (prefilter off) is never a reject; thr_sq = -inf (a
// beam the packet rejects, or past the tile's end) is always one (tn^2 is finite: the lanes and
// beams involved have finite coordinates).  A zero-length segment (au = 0, q = 0) has tn = 0 and is
// never rejected by a finite positive thr_sq.  Lanes off the tile are masked by the caller.
// Returned as the wave's lane mask of pairs to keep: each compare's ballot is the compare's own
// result mask, combined on the scalar unit (no bool materialisation in VALU).  All lanes must call.
__device__ __forceinline__ unsigned long long scan_keep_mask(const ScanLane &S, f3 au, const ScanStaged &B) {
    const float c = __builtin_fmaf(au.x, B.bu.x, __builtin_fmaf(au.y, B.bu.y, au.z * B.bu.z));
    const float u = __builtin_fmaf(-c, c, B.uc);
    const float x = __builtin_fmaf(au.x, B.m0.x, __builtin_fmaf(au.y, B.m0.y, au.z * B.m0.z));
    const float t = __builtin_fmaf(-B.bu.x, S.q.x, __builtin_fmaf(-B.bu.y, S.q.y, __builtin_fmaf(-B.bu.z, S.q.z, x)));
    return ~(__ballot(u >= 0.0101f) & __ballot((t * t) > B.thr_sq * u));
}

constexpr int kTileBlock = 64;   // one wave per workgroup: a finished wave frees its slot at once
constexpr int kQueueCap = 192;   // >= 63 left over + 128 appended by one scan step (two beams)

// One queued (beam, lane) pair: the beam's index in BVH order and the segment's lane.
struct QEntry {
    int32_t beam;
    int32_t lane;
};

struct TileShared {
    float4 tile[64][2];          // scan layout of the current leaf tile: (bu, Ab'), (m0, -)
    float4 acc[64];              // per-segment RGB sums and contribution count (w, exact below 2^24)
    unsigned long long rkm[64];  // exact batch: per-segment masks of its contributing positions (rank)
    QEntry q[kQueueCap + 64];    // prefilter survivors [0, t1), then one discard slot per lane
    int32_t stk[kStackDepth];
};

// The exact stage for n queued prefilter survivors q[first, first + n) (one per lane; all lanes
// call): the reference's box test on the beam's (group) box, then ComputeClosestPoints + kernel.
// The pair's segment comes from its SegRec, the beam line from L2.
__device__ __forceinline__ void tile_exact(TileShared &sh, int first, int n, const SegRec *__restrict__ srec,
                                           const float *__restrict__ sd, int64_t seg0,
                                           const BeamRec *__restrict__ recs, const float4 *__restrict__ pw,
                                           const BeamSet &bset, float R, float inv_maxd,
                                           bool count, const Lane &L) {
    const int lane = threadIdx.x & 63;
    const bool on = lane < n;
    const QEntry e = sh.q[first + (on ? lane : 0)];  // off lanes (a partial batch) read a valid entry
    const int sl = e.lane;
    const int64_t b = e.beam;
    // every load of the pair is issued at once (one memory round trip per batch; most queued pairs
    // pass the box test, so the second half is rarely wasted)
    const float4 *sr = seg_plane(srec, seg0 + sl, 0);  // packet-plane layout: plane k at sr[64 k]
    const float4 *rb = reinterpret_cast<const float4 *>(recs + b);
    (void)L;
    (void)sr;
    // SegRec plane k of this packet at byte (seg0 / 64) * 4096 + k * 1024 + sl * 16 (packet-plane layout;
    // one launch's records stay far below 4 GiB: bre_api.hip caps a launch's segments).  The beam
    // record and power stay 64-bit pointer loads: a beam index may exceed 2^26 (2^28) records of 64
    // (16) bytes, past a 32-bit byte offset.
    const __amdgpu_buffer_rsrc_t srs = buf_rsrc(srec);
    const unsigned int so_ = (unsigned int)(seg0 >> 6) << 12, vo = (unsigned int)sl << 4;
    const float4 s0 = buf_f4(srs, vo, so_), s3 = buf_f4(srs, vo + 3072u, so_), bx = rb[0], by = rb[1];
    // au = (p - o) * RN(1 / |A|), load_lane's own operations with the reciprocal k_seg_prep stored in
    // plane 3 (bit-identical to plane 2, which is not loaded: VALU for one of the pair's eight vector
    // loads -- the texture-data path is the kernel's busiest unit -- without a division per pair).
    // Plane 1's w is |A| with the sign bit carrying has_inf.
    const float4 s1 = buf_f4(srs, vo + 1024u, so_), bz = rb[2], bw = rb[3];
    const float mag_a = fabsf(s1.w);
    const f3 au_ = (mag_a != 0.0f) ? scale3(sub3(mk(s1.x, s1.y, s1.z), mk(s0.x, s0.y, s0.z)), s3.w) : mk(0.f, 0.f, 0.f);
    const float4 s2 = make_float4(au_.x, au_.y, au_.z, 0.f);
    // a uniform-radius set's power is in the record's last three words (BeamRec): seven loads per pair
    const float4 pv = bset.uniform ? make_float4(bw.y, bw.z, bw.w, 0.f) : pw[b];
    // phase 1: the box test (segment o, tmax, 1/d; the beam's box)
    const f3 o = mk(s0.x, s0.y, s0.z);
    const float tmax = s0.w;
    const Box6 box{bx.x, bx.y, bx.z, bx.w, by.x, by.y};
    float te;
    bool hit = on & node_test(box, o, mk(s3.x, s3.y, s3.z), tmax, te);
    const bool inf = __builtin_signbit(s1.w) != 0;  // has_inf, the sign of plane 1's |A|
    if (__ballot(on & inf) != 0ull) {
        if (on & inf) {
            // the rare axis-parallel ray: the literal slab test on its exact 1/d
            const int64_t so = seg0 + sl;
            const f3 d = mk(sd[3 * so], sd[3 * so + 1], sd[3 * so + 2]);
            const f3 inv = mk(1 / d.x, 1 / d.y, 1 / d.z);
            hit = slab_test(box, o, inv, inv.x < 0, inv.y < 0, inv.z < 0, tmax, nullptr);
        }
    }
    if (__ballot(hit) == 0ull) return;
    // phase 2: closest points + kernel
    float4 v = make_float4(0.f, 0.f, 0.f, 1.f);
    bool contrib = false;
    if (hit) {
        const float maxd = R + beam_radius(bset, bw.y);  // MaxDistance = currentBeamRadius + beam->radius
        float d2, unused;
        const bool ok = closest_distance_t<false, true>(o, mk(s1.x, s1.y, s1.z), mk(s2.x, s2.y, s2.z), mag_a,
                                                        mk(by.z, by.w, bz.x), mk(bz.y, bz.z, bz.w), bw.x, d2, unused);
        // |pA - pB| correctly rounded (photonbeam.cpp:500).  Without the compiler's small-input scaling
        // when maxd >= 2^-30: for d2 >= 2^-96 the root is bit-identical; below, both roots are < 2^-47.9,
        // so both pass dist < maxd and give r < 2^-17.9, r^2 < 2^-35 and 1 - r^2 == 1: the same value.
#if BRE_SQRT_NOSCALE
        const float dist = (maxd >= 0x1p-30f) ? sqrt_cr_noscale(d2) : sqrtf(d2);
#else
        const float dist = sqrtf(d2);
#endif
        if (ok & (dist < maxd)) {
            // r = dist / MaxDistance.  A uniform-radius set shares MaxDistance = R + radius over the
            // gather: the correctly rounded quotient from its reciprocal (div_by_shared, bit-identical to
            // the division; a quotient below 2^-126 gives r^2 = 0 and w = 1 either way)
            float rr;
            if (bset.uniform)
                rr = div_by_shared(dist, maxd, inv_maxd);
            else
                rr = dist / maxd;
            // 1 - fl(r^2) is 0 or >= 2^-24 (fl(r^2) <= 1 - 2^-24 unless it is 1): never in the scaled range
#if BRE_SQRT_NOSCALE
            const float w = sqrt_cr_noscale(1.0f - rr * rr);
#else
            const float w = sqrtf(1.0f - rr * rr);
#endif
            v.x = pv.x * w;
            v.y = pv.y * w;
            v.z = pv.z * w;
            contrib = true;
        }
    }
    // Accumulate into the segments' LDS sums in queue order, deterministically and without relying on
    // how the hardware orders same-address lanes of one instruction.  A pair's rank is the number of
    // its segment's contributing pairs below it in the batch (the mask bits below its lane): its
    // position among its segment's pairs in queue order.  Round k read-modify-writes the contributing rank-k
    // pairs, whose segments are distinct; one wave's LDS accesses are performed in order, so every
    // segment adds its terms in queue order.  A batch takes as many rounds as its most repeated segment
    // has pairs (up to 64 for a transposed tile's segment); round 3 took its ranks from ds_add_rtn_u32
    // and added ranks >= 8 by LDS float atomics, both of whose same-address orders within one
    // instruction are undocumented.  (`count` only decides whether the count is used: it is always kept.)
    (void)count;
    if (__ballot(contrib) == 0ull) return;
    // rank: every contributing lane ORs its bit into its segment's 64-bit mask with ds_or_rtn_b64, which
    // returns the mask as it was before this lane's OR.  Whatever order the hardware applies one
    // instruction's same-address lanes in, a lane's returned mask holds only lanes of its own segment;
    // if every returned mask holds only LOWER lanes, each segment's lanes were applied in ascending lane
    // order and the returned bit count is the lane's position among its segment's pairs in queue order.
    // That is checked (one ballot); a batch that fails it (never observed) takes its ranks from the
    // final masks instead, after the ORs.  Either way the rank is the lane-order position: the sums
    // are the same bits whatever the hardware's order.
    sh.rkm[lane] = 0ull;
    __builtin_amdgcn_wave_barrier();
    const unsigned long long lane_bit = 1ull << lane;
    unsigned long long before = 0ull;
    if (contrib) before = atomicOr(&sh.rkm[sl], lane_bit);
    int rank = contrib ? __popcll(before) : 64;
    // (a lane's own bit is never in its returned mask: a set bit at or above it means a higher lane went first)
    if (__ballot(contrib && (before >> lane) != 0ull) != 0ull) {
        __builtin_amdgcn_wave_barrier();
        rank = contrib ? lanes_below(sh.rkm[sl]) : 64;
    }
    // ranks are dense per segment (0 .. its count - 1): the first rank level no lane holds ends the rounds
    const auto round_k = [&](int k) {
        if (rank == k) {
            float4 a = sh.acc[sl];
            a.x += v.x;
            a.y += v.y;
            a.z += v.z;
            a.w += v.w;
            sh.acc[sl] = a;
        }
    };
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        if (__ballot(rank == k) == 0ull) return;
        round_k(k);
    }
    // a segment repeated more than 8 times in the batch (a transposed tile, few lanes on): the further
    // rounds, in a loop
#pragma nounroll
    for (int k = 8; k < 64; ++k) {
        if (__ballot(rank == k) == 0ull) return;
        round_k(k);
    }
}

// COUNT: also box-test every beam of every visited tile and count the candidates (the reference's
// C), plus traversal statistics; the queue of pairs and hence every sum are the same as without.
// pcnt (runtime, wave-uniform): count the contributions per segment in the production
// instantiation, with the production control flow (per-subtree counts in pcnt[.][1]).
template <bool COUNT, int MINW>
__global__ __launch_bounds__(kTileBlock, MINW) void k_gather_tile(
    int64_t nseg, const float *__restrict__ so, const float *__restrict__ sp_, const float *__restrict__ sd,
    const float *__restrict__ stmax, const SegRec *__restrict__ srec, float R, float *__restrict__ partial,
    int32_t *__restrict__ pcnt, const BeamRec *__restrict__ recs, const float4 *__restrict__ pw, BeamSet bset,
    const Node *__restrict__ nodes, const Node4 *__restrict__ nodes4, int64_t nvalid, int leaf_size,
    const int32_t *__restrict__ roots, int S, DevCounters *ctr, int stack_cap, int prefilter, int map, int tscan,
    int margin, const TileAxis *__restrict__ tax) {
    __shared__ TileShared shm[kTileBlock / 64];
    // Block -> (subtree, packet group).  map 1: block b works on packet group b / S and subtree
    // (b + b / S) mod S, so under the round-robin dispatch over the 8 XCDs every XCD sees every
    // subtree (balanced however unequal the subtrees are).  map 0: blocks b and b+8 share an XCD,
    // so for S >= 8 XCD (b & 7) is given the S/8 consecutive work roots below one depth-3 node (its
    // L2 serves one eighth of the tree).  Speed only, never correctness.
    int sub;
    int64_t grp;
    if (map == 3) {
        // LPT: all packets on the largest subtree (roots are sorted by size), then the next, ...
        const unsigned P = gridDim.x / (unsigned)S;
        grp = blockIdx.x % P;
        sub = (int)(blockIdx.x / P);
    } else if (map == 1) {
        grp = blockIdx.x / (unsigned)S;
        sub = (int)((blockIdx.x % (unsigned)S + grp) % (unsigned)S);
    } else if (map == 2 || S < 8) {
        sub = (int)(blockIdx.x % (unsigned)S);
        grp = blockIdx.x / (unsigned)S;
    } else {
        const unsigned per = (unsigned)S >> 3;
        const unsigned q = blockIdx.x >> 3;
        sub = (int)((blockIdx.x & 7u) * per + q % per);
        grp = q / per;
    }
    if (sub >= roots[S]) return;  // fewer work roots than S (small trees): whole block exits
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    wave_time(0, lane);
    TileShared &sh = shm[w];
    const int64_t s = grp * kTileBlock + threadIdx.x;
    const int64_t seg0 = grp * kTileBlock + (int64_t)__builtin_amdgcn_readfirstlane(w) * 64;  // lane 0 of this wave
    const bool count_c = COUNT || pcnt != nullptr;  // wave-uniform
    Lane L;
    const bool valid = load_lane(s, nseg, so, sp_, sd, stmax, L);
    Bundle K;
    K.delta = FLT_MAX;
    K.gbox = FLT_MAX;
    if (prefilter && __ballot(valid) != 0ull) K = make_bundle(L, valid);
    const ScanLane SL = make_scan_lane(L, margin);
    // the largest lane margin Al' of the packet, folded into every beam's threshold at staging (a
    // zero-length segment, Al' = FLT_MAX, is never rejected anyway: see scan_need)
    const float al_max = uniform_f(wave_max(valid && SL.al < FLT_MAX ? SL.al : 0.f));
    // 1 / MaxDistance of a uniform-radius set, correctly rounded, once per wave (tile_exact)
    const float inv_maxd = bset.uniform ? uniform_f(1.0f / (R + bset.radius)) : 0.f;
    sh.acc[lane] = make_float4(0.f, 0.f, 0.f, 0.f);
    __builtin_amdgcn_wave_barrier();
    int cand = 0;
    unsigned long long visits = 0;
    Prof pf;
    int t1 = 0;                // wave-uniform queue length: survivors in q[0, t1)
    int64_t cur_first = 0;     // first beam of the current leaf
    unsigned long long ph_stage = 0, ph_scan = 0, ph_exact = 0;
    unsigned long long ss_on = 0, ss_kept = 0, ss_steps = 0, ss_pairs = 0, ss_leaves = 0, ss_q = 0, ss_min = 0,
                       ss_tr = 0;
    const unsigned long long ph_t0 = phase_clock();

    // queue the (beam, lane) survivors of beam j of the current leaf, in lane order: every lane
    // stores (branch-free), a lane that queues nothing into its own discard slot
    // (m: the wave-uniform lane mask of the entries to queue)
    const int discard = kQueueCap + lane;
    const auto push = [&](unsigned long long m, int32_t e_beam, int32_t e_lane) {
        if (m == 0ull) return;
        int rank = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                  __builtin_amdgcn_mbcnt_lo((unsigned)m, (unsigned)t1));
        // computed by every lane (an opaque use keeps the compiler from sinking it under an exec mask),
        // then slot = lane in m ? rank : discard with the scalar mask itself as the select's condition
        // (inverse ballot): one v_cndmask, every lane stores
        asm volatile("" : "+v"(rank));
        const int slot = __builtin_amdgcn_inverse_ballot_w64(m) ? rank : discard;
        sh.q[slot] = QEntry{e_beam, e_lane};
        t1 += __popcll(m);
        if (COUNT) pf.queued += __popcll(m);
        if (BRE_SCAN_STATS) ss_q += __popcll(m);
    };
    // run the exact stage on every full batch of 64 queued pairs (the one call site in the scan),
    // then move the < 64 left over to the front of the queue
    const auto drain = [&]() {
        if (t1 < 64) return;
        __builtin_amdgcn_wave_barrier();
        const unsigned long long d0 = BRE_PHASE_TIMING ? phase_clock() : 0ull;
        int h = 0;
        while (t1 - h >= 64) {
            if (COUNT && lane == 0) ++pf.ccp_waves;
            tile_exact(sh, h, 64, srec, sd, seg0, recs, pw, bset, R, inv_maxd, count_c, L);
            if (!COUNT) pf.queued += 64;  // the production queue's length (counted per batch)
            h += 64;
            __builtin_amdgcn_wave_barrier();
        }
        const int rest = t1 - h;  // h >= 64 > rest: source and destination do not overlap
        if (rest > 0) {
            QEntry e{0, 0};
            if (lane < rest) e = sh.q[h + lane];
            __builtin_amdgcn_wave_barrier();
            if (lane < rest) sh.q[lane] = e;
            __builtin_amdgcn_wave_barrier();
        }
        t1 = rest;
        if (BRE_PHASE_TIMING) ph_exact += phase_clock() - d0;
    };

    // scan one leaf tile (<= 64 beams): lane j stages beam j's scan values in LDS; bundle rejects;
    // per lane the separable prefilter on the kept beams; survivors queue for the exact stage
    const auto leaf = [&](int32_t c, unsigned long long onm) {
        bool lane_on = ((onm >> lane) & 1ull) != 0ull;
        const int64_t first = (int64_t)(~c) * leaf_size;
        const int nb = (int)min((int64_t)leaf_size, nvalid - first);
        if (COUNT) {
            ++pf.leaves;
            pf.beams += nb;
        }
        if (!COUNT && tax != nullptr) {
            // the per-lane tile line reject: lanes whose segment line is too far from the tile's axis
            // line leave the tile; a tile no lane keeps is skipped before it is staged
            const float4 *tq = reinterpret_cast<const float4 *>(tax + (int64_t)(~c));
            const float4 ta = tq[0], tb = tq[1];
            if (tb.w < 0.f) return;
            ScanStaged A;
            A.bu = mk(ta.x, ta.y, ta.z);
            A.m0 = mk(tb.x, tb.y, tb.z);
            const float thr = ta.w + al_max;
            A.thr_sq = thr < FLT_MAX ? thr * thr : INFINITY;
            A.uc = 1.0001f;
            onm &= scan_keep_mask(SL, L.au, A);
            if (onm == 0ull) return;
            lane_on = ((onm >> lane) & 1ull) != 0ull;
        }
        const unsigned long long l0 = phase_clock();
        cur_first = first;
        ScanBeam T;
        T.bu = T.m0 = mk(0.f, 0.f, 0.f);
        T.ab = 0.f;
        bool keep = false;
        if (lane < nb) {
            // raised wave priority while the tile's records are requested: its loads issue ahead of
            // the other waves' scan VALU (round 5: C2 +0.3%, C3 +0.5%, profiles/r5/run27; the same
            // around the exact stage's loads measured -0.1%)
            __builtin_amdgcn_s_setprio(2);
            const BeamV r = load_beam(recs, first + lane, bset);
            T = make_scan_beam(r, R, margin);
            __builtin_amdgcn_s_setprio(0);
            // packet-level rejects (see make_bundle, bundle_box_miss): a beam far from every segment
            // of the packet, or whose box no lane's ray can reach, is skipped by all lanes
            keep = !prefilter ||
                   !((margin ? bundle_far_sep(K, r.b0, T.bu, T.m0, R + r.radius, r.mag_b)
                             : bundle_far(K, r.b0, r.bu, R + r.radius, 0)) ||
                     bundle_box_miss(K, r.box));
        }
        const unsigned long long all = nb >= 64 ? ~0ull : ((1ull << nb) - 1ull);
        const unsigned long long km = __ballot(keep) & all;
        __builtin_amdgcn_wave_barrier();  // the previous tile's reads are done
        // every lane writes (the transposed scan reads record `lane`): thr_sq = -inf for a beam the
        // packet rejects or past the tile's end (bu = m0 = 0), which scan_need always rejects; +inf
        // with the prefilter off (never a reject)
        const float thr = T.ab + al_max;
        const float thr_sq = !keep ? -INFINITY : (prefilter ? thr * fabsf(thr) : INFINITY);
        sh.tile[lane][0] = make_float4(T.bu.x, T.bu.y, T.bu.z, thr_sq);
        sh.tile[lane][1] = make_float4(T.m0.x, T.m0.y, T.m0.z, 1.0001f);
        __builtin_amdgcn_wave_barrier();
        if (COUNT) {
            pf.useful += __popcll(km);
            // every beam of the tile: the reference box test (candidates) and the pairs the
            // prefilters drop; the queue gets exactly the production survivors, in order
            for (int j = 0; j < nb; ++j) {
                const bool kept = (km >> j) & 1ull;
                const unsigned long long mk_ = scan_keep_mask(SL, L.au, scan_beam_lds(sh.tile, j)) & onm;
                const bool need = kept && ((mk_ >> lane) & 1ull);
                const Box6 box = load_beam(recs, first + j, bset).box;
                float te;
                bool hit = lane_on & node_test(box, L.o, L.invs, L.tmax, te);
                if (L.has_inf) hit = lane_on & slab_test(box, L.o, L.inv, L.n0, L.n1, L.n2, L.tmax, nullptr);
                cand += hit;
                pf.rejects += hit & !need;
                if (kept) push(mk_, (int32_t)(cur_first + j), lane);
                drain();
            }
            return;
        }
        const unsigned long long l1 = phase_clock();
        if (BRE_PHASE_TIMING) ph_stage += l1 - l0;
        const unsigned long long ex0 = ph_exact;
        // Few lanes on the tile and many kept beams: the TRANSPOSED scan, one on-lane segment per step
        // against all kept beams at once (lane j: beam j), so a tile costs min(on lanes, kept beams)
        // steps.  Segment i's pairs are queued in beam order, exactly the order the beam-major scan
        // gives them, and every sum is a per-segment sum in queue order: bit-identical results.  The
        // batches then hold long stretches of one segment, which the exact stage adds in as many
        // read-modify-write rounds, in queue order.
        const bool transposed = tscan > 0 && __popcll(onm) * 8 < __popcll(km) * tscan;
        if (BRE_SCAN_STATS) {
            const unsigned long long on = __popcll(onm), kp = __popcll(km);
            ss_on += on;
            ss_kept += kp;
            ss_steps += transposed ? on : (kp + 1) / 2;
            ss_pairs += (on * kp + 63) / 64;
            ss_min += on < kp ? on : kp;
            ss_tr += transposed;
            ++ss_leaves;
        }
        if (transposed) {
            // lane j: beam j (Ab' = -inf staged for a beam the packet rejects), segment i on the tile
            unsigned long long rest = onm;
            // two on-lane segments per step (independent readlanes and tests: ILP), queued in order
            while (rest != 0ull) {
                const int i1 = __ffsll((long long)rest) - 1;
                rest &= rest - 1ull;
                const bool two = rest != 0ull;
                const int i2 = two ? __ffsll((long long)rest) - 1 : i1;
                if (two) rest &= rest - 1ull;
                ScanLane S1, S2;
                S1.q = mk(readlane_f(SL.q.x, i1), readlane_f(SL.q.y, i1), readlane_f(SL.q.z, i1));
                S2.q = mk(readlane_f(SL.q.x, i2), readlane_f(SL.q.y, i2), readlane_f(SL.q.z, i2));
                S1.al = S2.al = 0.f;
                const f3 au1 = mk(readlane_f(L.au.x, i1), readlane_f(L.au.y, i1), readlane_f(L.au.z, i1));
                const f3 au2 = mk(readlane_f(L.au.x, i2), readlane_f(L.au.y, i2), readlane_f(L.au.z, i2));
                // & km: a beam the packet rejected (thr_sq = -inf) still passes scan_keep_mask when it
                // is near-parallel to segment i (u < 0.0101); the beam-major scan never visits it
                const ScanStaged Bl = scan_beam_lds(sh.tile, lane);
                const unsigned long long n1 = scan_keep_mask(S1, au1, Bl) & km;
                const unsigned long long n2 = scan_keep_mask(S2, au2, Bl) & km;
                push(n1, (int32_t)(cur_first + lane), i1);
                if (two) push(n2, (int32_t)(cur_first + lane), i2);
                drain();
            }
            if (BRE_PHASE_TIMING) ph_scan += (phase_clock() - l1) - (ph_exact - ex0);
            return;
        }
        // two kept beams per step: independent reads and prefilters (ILP), then the survivors are
        // queued beam by beam in order
        unsigned long long todo = km;
        while (todo != 0ull) {
            const int j1 = __ffsll((long long)todo) - 1;
            todo &= todo - 1ull;
            const bool two = todo != 0ull;
            const int j2 = two ? __ffsll((long long)todo) - 1 : j1;
            if (two) todo &= todo - 1ull;
            const ScanStaged B1 = scan_beam_lds(sh.tile, j1), B2 = scan_beam_lds(sh.tile, j2);
            // lane masks: every lane evaluates both tests, the lanes off the tile are masked out
            const unsigned long long n1 = scan_keep_mask(SL, L.au, B1) & onm;
            const unsigned long long n2 = scan_keep_mask(SL, L.au, B2) & onm;
            push(n1, (int32_t)(cur_first + j1), lane);
            if (two) push(n2, (int32_t)(cur_first + j2), lane);
            drain();
        }
        if (BRE_PHASE_TIMING) ph_scan += (phase_clock() - l1) - (ph_exact - ex0);
    };

    if (__ballot(valid) != 0ull) {
        // Fixed-order walk of the 4-wide view (Node4): a visit tests the four grandchild boxes of a
        // binary node; the leaf tiles it finds are scanned, in slot order, before the walk goes on
        // with the lowest-slot internal child, the others stacked.  (The gather has no early exit, so
        // any order finds every pair; a fixed one keeps the queue order a function of the tree.)
        const int32_t root = roots[sub];
        int32_t pc0 = 0, pc1 = 0, pc2 = 0, pc3 = 0;  // pending leaf tiles, in slot order
        unsigned long long pm0 = 0ull, pm1 = 0ull, pm2 = 0ull, pm3 = 0ull;  // lanes on each one's box
        int npend = 0;
        int node = root;
        bool have_node = root >= 0;
        if (!have_node) {
            pc0 = root;
            pm0 = __ballot(valid);
            npend = 1;
        }
        int sp = 0;
        while (true) {
#pragma nounroll
            for (; npend > 0; --npend) {
                leaf(pc0, pm0);
                pc0 = pc1;
                pm0 = pm1;
                pc1 = pc2;
                pm1 = pm2;
                pc2 = pc3;
                pm2 = pm3;
            }
            if (!have_node) {
                if (sp == 0) break;
                --sp;
                node = sh.stk[sp];
            }
            node = __builtin_amdgcn_readfirstlane(node);
            if (COUNT) ++visits;
            const Node4 *nq = nodes4 + node;
            int32_t nxt = 0;
            have_node = false;
            bool ovf = false;
            // slots high to low: a leaf goes to the FRONT of the pending list and an internal child
            // becomes the next node (the one it replaces is stacked), so both end in slot order
#pragma unroll
            for (int k = 3; k >= 0; --k) {
                const int32_t ck = nq->child[k];
                const Box6 bk{nq->lo[0][k], nq->lo[1][k], nq->lo[2][k], nq->hi[0][k], nq->hi[1][k], nq->hi[2][k]};
                float te;
                const bool h = valid & (ck != kEmptyChild) & node_test(bk, L.o, L.invs, L.tmax, te);
                const unsigned long long m = __ballot(h);
                if (m != 0ull) {
                    if (ck < 0) {
                        pc3 = pc2;
                        pm3 = pm2;
                        pc2 = pc1;
                        pm2 = pm1;
                        pc1 = pc0;
                        pm1 = pm0;
                        pc0 = ck;
                        pm0 = m;
                        ++npend;
                    } else {
                        if (have_node) {
                            if (sp >= stack_cap) {
                                ovf = true;
                            } else {
                                sh.stk[sp] = nxt;
                                ++sp;
                            }
                        }
                        nxt = ck;
                        have_node = true;
                    }
                }
            }
            if (ovf) {
                // never silent: the host turns the flag into BRE_ERR_STATE (bre_api.hip)
                if (lane == 0) atomicOr(&ctr->flags, kFlagStack);
                break;
            }
            node = nxt;
        }
        // drain the prefilter survivors
        __builtin_amdgcn_wave_barrier();
        if (t1 > 0) {
            if (COUNT && lane == 0) ++pf.ccp_waves;
            tile_exact(sh, 0, t1, srec, sd, seg0, recs, pw, bset, R, inv_maxd, count_c, L);
            if (!COUNT) pf.queued += (unsigned long long)t1;
        }
        t1 = 0;
    }
    __builtin_amdgcn_wave_barrier();
    if (valid) {
        float *dst = partial + 3 * ((int64_t)sub * nseg + s);
        const float4 a = sh.acc[lane];
        dst[0] = a.x;
        dst[1] = a.y;
        dst[2] = a.z;
        if (count_c) {
            pcnt[2 * ((int64_t)sub * nseg + s)] = COUNT ? cand : -1;
            pcnt[2 * ((int64_t)sub * nseg + s) + 1] = (int32_t)a.w;
        }
    }
    wave_time(1, lane);
    // the production instantiation's own queue length (contribution counting on): what its exact stage ran
    if (!COUNT && !BRE_SCAN_STATS && !BRE_PHASE_TIMING && count_c && lane == 0 && pf.queued != 0ull)
        atomicAdd(&ctr->queued_pairs, pf.queued);
    if (BRE_SCAN_STATS && !COUNT && lane == 0) {
        atomicAdd(&ctr->candidates, ss_on);
        atomicAdd(&ctr->contributions, ss_kept);
        atomicAdd(&ctr->node_visits, ss_steps);
        atomicAdd(&ctr->leaf_visits, ss_pairs);
        atomicAdd(&ctr->beam_evals, ss_leaves);
        atomicAdd(&ctr->useful_beam_evals, ss_q);
        atomicAdd(&ctr->prefilter_rejects, ss_min);
        atomicAdd(&ctr->ccp_wave_evals, ss_tr);
    }
    if (BRE_PHASE_TIMING && !COUNT && lane == 0) {
        atomicAdd(&ctr->candidates, ph_stage);
        atomicAdd(&ctr->contributions, ph_scan);
        atomicAdd(&ctr->node_visits, ph_exact);
        atomicAdd(&ctr->leaf_visits, phase_clock() - ph_t0);
    }
    if (COUNT) {
        unsigned long long rj = pf.rejects;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) rj += __shfl_xor(rj, off);
        if (lane == 0) {
            atomicAdd(&ctr->node_visits, visits);
            atomicAdd(&ctr->leaf_visits, pf.leaves);
            atomicAdd(&ctr->beam_evals, pf.beams);
            atomicAdd(&ctr->useful_beam_evals, pf.useful);
            atomicAdd(&ctr->prefilter_rejects, rj);
            atomicAdd(&ctr->ccp_wave_evals, pf.ccp_waves);
            atomicAdd(&ctr->queued_pairs, pf.queued);
        }
    }
}

// One 64-B record per gathered segment for the tile kernel's exact stage (see SegRec, packet-plane
// layout): the values load_lane derives, computed once per gather instead of once per (packet,
// subtree) wave.
__global__ __launch_bounds__(kPassBlock) void k_seg_prep(int64_t nseg, const float *__restrict__ so,
                                                  const float *__restrict__ sp_, const float *__restrict__ sd,
                                                  const float *__restrict__ stmax, SegRec *__restrict__ out) {
    const int64_t s = (int64_t)blockIdx.x * kPassBlock + threadIdx.x;
    if (s >= nseg) return;
    Lane L;
    load_lane(s, nseg, so, sp_, sd, stmax, L);
    float4 *q = const_cast<float4 *>(seg_plane(out, s, 0));  // packet-plane layout (bre_device.h)
    q[0] = make_float4(L.o.x, L.o.y, L.o.z, L.tmax);
    // |A| >= 0: its sign bit carries has_inf; plane 3's w is RN(1 / |A|) (0 for a zero-length segment),
    // the reciprocal div3 forms in load_lane, so the exact stage recomputes au without a division
    q[64] = make_float4(L.p.x, L.p.y, L.p.z, L.has_inf ? -L.mag_a : L.mag_a);
    q[128] = make_float4(L.au.x, L.au.y, L.au.z, __int_as_float(L.has_inf ? 1 : 0));
    q[192] = make_float4(L.invs.x, L.invs.y, L.invs.z, L.mag_a != 0.0f ? 1.0f / L.mag_a : 0.0f);
}

// Sum the per-subtree partials of each segment in subtree order; write seg_rgb and add the
// segment's sum to its pixel (one float atomic per channel, PhotonBeamPixel::Ld +=).  With counts,
// also sum the per-subtree candidate / contribution counts (candidates -1: not counted).  seg_index
// (optional) maps the gathered order to the caller's order of seg_rgb / seg_counts.
__global__ __launch_bounds__(kPassBlock) void k_reduce(int64_t nseg, const float *__restrict__ partial,
                                                const int32_t *__restrict__ pcnt, const int32_t *__restrict__ roots,
                                                int S, const int32_t *__restrict__ pixel, int64_t npix,
                                                float *__restrict__ accum, float *__restrict__ seg_rgb,
                                                int32_t *__restrict__ seg_counts, const int32_t *__restrict__ seg_index,
                                                DevCounters *ctr) {
    const int64_t s = (int64_t)blockIdx.x * kPassBlock + threadIdx.x;
    const bool in = s < nseg;
    const int nr = roots[S];
    float cr = 0.f, cg = 0.f, cb = 0.f;
    long long c = 0, k = 0;
    if (in) {
        for (int j = 0; j < nr; ++j) {
            const float *q = partial + 3 * ((int64_t)j * nseg + s);
            cr += q[0];
            cg += q[1];
            cb += q[2];
            if (pcnt) {
                c += pcnt[2 * ((int64_t)j * nseg + s)];
                k += pcnt[2 * ((int64_t)j * nseg + s) + 1];
            }
        }
        const int64_t so = seg_index ? (int64_t)seg_index[s] : s;
        if (seg_rgb) {
            seg_rgb[3 * so] = cr;
            seg_rgb[3 * so + 1] = cg;
            seg_rgb[3 * so + 2] = cb;
        }
        if (seg_counts) {
            seg_counts[2 * so] = c < 0 ? -1 : (int32_t)c;
            seg_counts[2 * so + 1] = (int32_t)k;
        }
        if (accum) {
            const int32_t px = pixel[s];
            if (px < 0 || px >= npix) {
                atomicOr(&ctr->flags, kFlagPixel);
            } else if (cr != 0.f || cg != 0.f || cb != 0.f) {
                atomicAdd(&accum[3 * (int64_t)px], cr);
                atomicAdd(&accum[3 * (int64_t)px + 1], cg);
                atomicAdd(&accum[3 * (int64_t)px + 2], cb);
            }
        }
    }
    if (pcnt) {
        unsigned long long uc = c > 0 ? (unsigned long long)c : 0ull, uk = (unsigned long long)k;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            uc += __shfl_xor(uc, off);
            uk += __shfl_xor(uk, off);
        }
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(&ctr->candidates, uc);
            atomicAdd(&ctr->contributions, uk);
        }
    }
}

// Work roots: the BVH frontier at depth log2(S) (leaves above it stay in the frontier), ordered by the
// number of leaf tiles below each root, largest first (stable): with block map 3 every packet's
// waves on the largest subtrees are dispatched first and the kernel's tail is made of small ones.
// The leaves below a Karras node are a contiguous range (bre_build.hip), found by its leftmost and
// rightmost descents.  The partial sums are added in this root order (k_reduce): deterministic.
//
// Starting from the root, the frontier's LARGEST internal node (leaf tiles below it, Node::nleaf; ties:
// the lowest frontier position) is replaced by its children (the first in its place, the second
// appended) while the frontier stays within S entries, so the S work roots are as equal in size as
// the tree allows: the longest (packet, subtree) waves, which end the launch, are as short as they can
// be (a breadth-first frontier left subtrees of very unequal size, and an emulated 1/8 rank's
// iteration-0 gather 37% above 1/8 of N = 1's).  Then the roots are ordered largest first (ties in
// frontier order) for the LPT block map.
//
// The greedy loop is serial (up to S - 1 expansions: 0.39 ms at C2 as a block-wide reduction per
// expansion), but its result is not: every expanded node has more leaf tiles than its children, so
// the expansions come in decreasing order of size and the expanded set E is the S - 1 largest
// interior nodes (fewer when the tree has fewer), a subtree from the root; the roots are E's children
// outside E.  So, with all threads:
//   1. cache, breadth first, every interior node with at least total / S leaf tiles (the frontier
//      partitions the total over <= S entries, so its largest entry, the only one ever expanded, has
//      at least total / S): its leaf tiles, children, their leaf tiles and cache slots;
//   2. E = the S - 1 cached nodes of largest (leaf tiles, -index), each ranked against all others;
//   3. the roots: E's children outside E (the whole tree's root when S = 1);
//   4. ranks: leaf tiles descending, ties by child index.
// Ties of equal size are broken by node index instead of the frontier position the serial form used
// (any frontier is a valid split; this one is deterministic).  A cache overflow (never seen: C2 caches
// ~600 of 4096 slots at S = 256) still yields a valid split: the cached nodes form a subtree from the
// root, so E's top-(S - 1) choice among them is one too.
constexpr int kRootSlots = 4096;
// the cache, in global scratch (one wave computes the roots: a one-wave workgroup with no LDS fits a
// concurrent gather's slots, bre_slot.hip; round 5's version kept it in 140 KB of LDS, a whole CU)
struct RootsScratch {
    int32_t id[kRootSlots];     // cached node
    int32_t nl[kRootSlots];     // its leaf tiles (Node::nleaf)
    int32_t ch[kRootSlots][2];  // its children
    int32_t cw[kRootSlots][2];  // their leaf tiles (1: a leaf tile, 0: empty)
    int32_t cs[kRootSlots][2];  // their cache slots (-1: not cached)
    int32_t in_e[kRootSlots];
    int32_t fc[kMaxSplit + 1], fw[kMaxSplit + 1];  // the roots, unordered
};

// children, parent and leaf tiles of node x: the record's last 16 bytes
__device__ __forceinline__ int4 node_tail(const Node *__restrict__ nodes, int32_t x) {
    return *reinterpret_cast<const int4 *>(&nodes[x].child[0]);
}

// the wave's own global writes visible to its later reads (device-scope release + acquire)
__device__ __forceinline__ void wave_sync_global() {
    __threadfence();
    __builtin_amdgcn_wave_barrier();
}

// key of a node or root of w leaf tiles and index x: larger first, ties by ascending (signed) index
__device__ __forceinline__ unsigned long long root_key(int32_t w, int32_t x) {
    return ((unsigned long long)(unsigned int)w << 32) | (0xffffffffu - ((unsigned int)x ^ 0x80000000u));
}

// rank of key kk among the n keys key(w[j], x[j]) (the number of larger ones): 64 keys per step, read by
// one lane each and broadcast by readlane
__device__ __forceinline__ int rank_among(const int32_t *w, const int32_t *x, int n, unsigned long long kk) {
    int rank = 0;
    for (int j0 = 0; j0 < n; j0 += 64) {
        const int j = j0 + (int)threadIdx.x;
        const unsigned long long kv = j < n ? root_key(w[j], x[j]) : 0ull;
        const int m = min(64, n - j0);
        for (int q = 0; q < m; ++q) {
            const unsigned long long kj =
                ((unsigned long long)(unsigned int)__builtin_amdgcn_readlane((int)(kv >> 32), q) << 32) |
                (unsigned int)__builtin_amdgcn_readlane((int)(unsigned int)kv, q);
            rank += kj > kk;
        }
    }
    return rank;
}

__global__ __launch_bounds__(64) void k_roots(const Node *__restrict__ nodes, int S, int32_t *__restrict__ roots,
                                              RootsScratch *__restrict__ g) {
    const int t = threadIdx.x;
    const unsigned long long below = (1ull << t) - 1ull;
    const int32_t total = nodes[0].nleaf;
    const int32_t heavy = total / S;
    if (t == 0) g->id[0] = 0;
    wave_sync_global();
    // 1. breadth-first cache of the heavy interior nodes (slots handed out in lane order per child)
    int cnt = 1, lo = 0, hi = 1;
    while (lo < hi) {
        for (int k0 = lo; k0 < hi; k0 += 64) {
            const int k = k0 + t;
            const bool act = k < hi;
            const int4 q = act ? node_tail(nodes, g->id[k]) : make_int4(kEmptyChild, kEmptyChild, 0, 0);
            const int32_t c[2] = {q.x, q.y};
            int32_t w[2];
            bool h[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                w[j] = c[j] == kEmptyChild ? 0 : (c[j] < 0 ? 1 : node_tail(nodes, c[j]).w);
                h[j] = act && c[j] >= 0 && w[j] >= heavy;
            }
            int32_t sl[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const unsigned long long m = __ballot(h[j]);
                const int s = cnt + __popcll(m & below);
                sl[j] = (h[j] && s < kRootSlots) ? s : -1;
                if (sl[j] >= 0) g->id[s] = c[j];
                cnt += __popcll(m);
            }
            if (act) {
                g->nl[k] = q.w;
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    g->ch[k][j] = c[j];
                    g->cw[k][j] = w[j];
                    g->cs[k][j] = sl[j];
                }
            }
        }
        wave_sync_global();
        lo = hi;
        hi = min(cnt, kRootSlots);
    }
    const int nc = min(cnt, kRootSlots);
    // 2. E: the S - 1 largest cached nodes
    for (int k0 = 0; k0 < nc; k0 += 64) {
        const int k = k0 + t;
        const unsigned long long kk = k < nc ? root_key(g->nl[k], g->id[k]) : ~0ull;
        const int rank = rank_among(g->nl, g->id, nc, kk);
        if (k < nc) g->in_e[k] = rank < S - 1;
    }
    wave_sync_global();
    // 3. the roots: E's children outside E (the whole tree's root when S = 1)
    int nf = 0;
    for (int k0 = 0; k0 < nc; k0 += 64) {
        const int k = k0 + t;
        const bool e = k < nc && g->in_e[k];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            int32_t c = kEmptyChild, s = -1;
            if (e) {
                c = g->ch[k][j];
                s = g->cs[k][j];
            }
            const bool root = e && c != kEmptyChild && !(s >= 0 && g->in_e[s]);
            const unsigned long long m = __ballot(root);
            if (root) {
                const int f = nf + __popcll(m & below);
                g->fc[f] = c;
                g->fw[f] = g->cw[k][j];
            }
            nf += __popcll(m);
        }
    }
    if (!g->in_e[0]) {
        if (t == 0) {
            g->fc[0] = 0;
            g->fw[0] = total;
        }
        nf = 1;
    }
    wave_sync_global();
    // 4. ranks: leaf tiles descending, ties by child index
    for (int k0 = 0; k0 < nf; k0 += 64) {
        const int k = k0 + t;
        const unsigned long long kk = k < nf ? root_key(g->fw[k], g->fc[k]) : ~0ull;
        const int rank = rank_among(g->fw, g->fc, nf, kk);
        if (k < nf) roots[rank] = g->fc[k];
    }
    for (int k = nf + t; k < S; k += 64) roots[k] = kEmptyChild;
    if (t == 0) roots[S] = nf;
}

template <bool COUNT>
__global__ __launch_bounds__(kThreadBlock) void k_gather_thread(
    int64_t nseg, const float *__restrict__ so, const float *__restrict__ sp_, const float *__restrict__ sd,
    const float *__restrict__ stmax, const int32_t *__restrict__ pixel, float R, int64_t npix,
    float *__restrict__ accum, float *__restrict__ seg_rgb, int32_t *__restrict__ seg_counts,
    const BeamRec *__restrict__ recs, const float4 *__restrict__ pw, BeamSet bset, const Node *__restrict__ nodes,
    int64_t nvalid, int leaf_size, DevCounters *ctr, int stack_cap) {
    __shared__ int32_t stk[kThreadStackDepth][kThreadBlock];
    const int tid = threadIdx.x;
    const int64_t s = (int64_t)blockIdx.x * kThreadBlock + tid;
    Lane L;
    const bool valid = load_lane(s, nseg, so, sp_, sd, stmax, L);
    float cr = 0.f, cg = 0.f, cb = 0.f;
    int cand = 0, contrib = 0;
    unsigned long long visits = 0;
    if (valid && nvalid > 0) {
        int node = 0;
        int sp = 0;
        const int cap = stack_cap < kThreadStackDepth ? stack_cap : kThreadStackDepth;
        while (true) {
            const NodeV n = load_node(nodes, node);
            if (COUNT) ++visits;
            const int32_t c0 = n.c0, c1 = n.c1;
            float te0 = 0.f, te1 = 0.f;
            bool h0 = (c0 != kEmptyChild) & node_test(n.b0, L.o, L.invs, L.tmax, te0);
            bool h1 = (c1 != kEmptyChild) & node_test(n.b1, L.o, L.invs, L.tmax, te1);
            if (h0 && c0 < 0) {
                const int64_t first = (int64_t)(~c0) * leaf_size;
                const int cnt = (int)min((int64_t)leaf_size, nvalid - first);
                for (int j = 0; j < cnt; ++j)
                    eval_beam<COUNT>(L, true, load_beam(recs, first + j, bset), pw, first + j, R, cr, cg, cb, cand, contrib);
                h0 = false;
            }
            if (h1 && c1 < 0) {
                const int64_t first = (int64_t)(~c1) * leaf_size;
                const int cnt = (int)min((int64_t)leaf_size, nvalid - first);
                for (int j = 0; j < cnt; ++j)
                    eval_beam<COUNT>(L, true, load_beam(recs, first + j, bset), pw, first + j, R, cr, cg, cb, cand, contrib);
                h1 = false;
            }
            if (h0 && h1) {
                const bool first0 = !(te1 < te0);
                if (sp >= cap) {
                    atomicOr(&ctr->flags, kFlagStack);
                    break;
                }
                stk[sp][tid] = first0 ? c1 : c0;
                ++sp;
                node = first0 ? c0 : c1;
            } else if (h0) {
                node = c0;
            } else if (h1) {
                node = c1;
            } else {
                if (sp == 0) break;
                --sp;
                node = stk[sp][tid];
            }
        }
    }
    finish_lane<COUNT>(s, valid, cr, cg, cb, cand, contrib, visits, pixel, npix, accum, seg_rgb, seg_counts, ctr);
}

__global__ void k_zero_seg(int64_t nseg, float *__restrict__ seg_rgb, int32_t *__restrict__ seg_counts,
                           const int32_t *__restrict__ seg_index) {
    const int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (i >= nseg) return;
    const int64_t s = seg_index ? (int64_t)seg_index[i] : i;  // the caller's entry of gathered segment i
    if (seg_rgb) {
        seg_rgb[3 * s] = 0.f;
        seg_rgb[3 * s + 1] = 0.f;
        seg_rgb[3 * s + 2] = 0.f;
    }
    if (seg_counts) {
        seg_counts[2 * s] = 0;
        seg_counts[2 * s + 1] = 0;
    }
}

}  // namespace

// The 4-wide view (Node4): one thread per binary node.  Slot order is the binary order (child 0's
// children, then child 1's), so a fixed-order walk of the 4-wide view visits the leaves in the same
// left-to-right order as a fixed-order binary walk.  A grandchild box lies inside its parent's box, so
// testing it directly prunes at least as tightly as testing both levels.
__global__ __launch_bounds__(64) void k_collapse4(const Node *__restrict__ nodes, int64_t nnodes,
                                                   Node4 *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (i >= nnodes) return;
    const Node &n = nodes[i];
    Node4 q;
    int k = 0;
    const auto put = [&](int32_t c, const float *lo, const float *hi) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            q.lo[a][k] = lo[a];
            q.hi[a][k] = hi[a];
        }
        q.child[k] = c;
        ++k;
    };
    for (int c = 0; c < 2; ++c) {
        const int32_t ch = n.child[c];
        if (ch == kEmptyChild) continue;
        if (ch >= 0) {
            const Node &m = nodes[ch];
            for (int d = 0; d < 2; ++d)
                if (m.child[d] != kEmptyChild) put(m.child[d], m.lo[d], m.hi[d]);
        } else {
            put(ch, n.lo[c], n.hi[c]);
        }
    }
    for (; k < 4; ++k) {
#pragma unroll
        for (int a = 0; a < 3; ++a) q.lo[a][k] = q.hi[a][k] = 0.f;
        q.child[k] = kEmptyChild;
    }
    q.pad[0] = q.pad[1] = q.pad[2] = q.pad[3] = 0;
    out[i] = q;
}

hipError_t launch_collapse4(const Node *nodes, int64_t nnodes, Node4 *out, hipStream_t s) {
    if (nnodes <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_collapse4, dim3((unsigned int)((nnodes + 63) / 64)), dim3(64), 0, s, nodes, nnodes, out);
    return hipGetLastError();
}

// A work-root shard's list: the roots rank, rank + count, ... of the size-ordered list (so every shard
// gets large and small subtrees), S2 entries padded with kEmptyChild, their number in out[S2].
__global__ void k_roots_shard(const int32_t *__restrict__ roots, int S, int rank, int count, int S2,
                              int32_t *__restrict__ out) {
    const int n = roots[S];
    const int n2 = n > rank ? (n - rank + count - 1) / count : 0;
    for (int k = threadIdx.x; k < S2; k += blockDim.x) out[k] = k < n2 ? roots[rank + k * count] : kEmptyChild;
    if (threadIdx.x == 0) out[S2] = n2;
}

hipError_t launch_roots_shard(const int32_t *roots, int S, int rank, int count, int S2, int32_t *out,
                              hipStream_t s) {
    hipLaunchKernelGGL(k_roots_shard, dim3(1), dim3(64), 0, s, roots, S, rank, count, S2, out);
    return hipGetLastError();
}

size_t roots_scratch_bytes() { return sizeof(RootsScratch); }

hipError_t launch_roots(const Node *nodes, int S, int32_t *roots, void *scratch, hipStream_t s) {
    hipLaunchKernelGGL(k_roots, dim3(1), dim3(64), 0, s, nodes, S, roots, static_cast<RootsScratch *>(scratch));
    return hipGetLastError();
}

hipError_t launch_gather(const GatherArgs &a, int kernel, bool counters, hipStream_t s) {
    if (a.nseg == 0) return hipSuccess;
    const int stack_cap = a.stack_cap > 0 ? a.stack_cap : kStackDepth;
    if (stack_cap > kStackDepth) return hipErrorInvalidValue;
    if (kernel == 2) {
        const dim3 grid((unsigned int)((a.nseg + kThreadBlock - 1) / kThreadBlock));
        int32_t *cnt = a.seg_index ? nullptr : a.seg_counts;
        float *rgb = a.seg_index ? nullptr : a.seg_rgb;
        if (a.seg_index && (a.seg_rgb || a.seg_counts)) return hipErrorInvalidValue;  // kernel 2 writes in place
        if (counters)
            hipLaunchKernelGGL(k_gather_thread<true>, grid, dim3(kThreadBlock), 0, s, a.nseg, a.o, a.p, a.d, a.tmax,
                               a.pixel, a.R, a.npix, a.accum, rgb, cnt, a.recs, a.pow, a.bset, a.nodes, a.nvalid,
                               a.leaf_size, a.ctr, stack_cap);
        else
            hipLaunchKernelGGL(k_gather_thread<false>, grid, dim3(kThreadBlock), 0, s, a.nseg, a.o, a.p, a.d, a.tmax,
                               a.pixel, a.R, a.npix, a.accum, rgb, cnt, a.recs, a.pow, a.bset, a.nodes, a.nvalid,
                               a.leaf_size, a.ctr, stack_cap);
        return hipGetLastError();
    }
    if (kernel != 4) return hipErrorInvalidValue;
    // per-subtree counts: candidates + contributions with counters, contributions alone otherwise
    int32_t *pcnt = (counters || a.seg_counts) ? a.pcnt : nullptr;
    if ((counters || a.seg_counts) && !pcnt) return hipErrorInvalidValue;
    if (!a.segrec || a.leaf_size > 64) return hipErrorInvalidValue;
    if (!a.nodes4) return hipErrorInvalidValue;  // the 4-wide walk needs the collapsed view
    hipLaunchKernelGGL(k_seg_prep, dim3((unsigned int)((a.nseg + kPassBlock - 1) / kPassBlock)), dim3(kPassBlock), 0, s, a.nseg, a.o, a.p, a.d,
                       a.tmax, a.segrec);
    const TileAxis *tax = nullptr;
    if (a.tileax && a.segbox && a.prefilter && a.nvalid > 0) {
        const int64_t ntiles = (a.nvalid + a.leaf_size - 1) / a.leaf_size;
        hipLaunchKernelGGL(k_segbox_init, dim3(1), dim3(64), 0, s, a.segbox);
        hipLaunchKernelGGL(k_segbox, dim3((unsigned int)std::min<int64_t>(kSegboxBlocks, (a.nseg + kPassBlock - 1) / kPassBlock)), dim3(kPassBlock), 0, s, a.nseg, a.o, a.p,
                           a.segbox);
        hipLaunchKernelGGL(k_tile_axis, dim3((unsigned int)ntiles), dim3(64), 0, s, a.recs, a.bset, a.nvalid,
                           a.leaf_size, a.segbox, a.R, a.tileax);
        tax = a.tileax;
    }
    const dim3 grid4((unsigned int)(((a.nseg + kTileBlock - 1) / kTileBlock) * a.split));
    // block map 0 deals S / 8 roots to each XCD: a split that is not a multiple of 8 (work-root shards:
    // ceil(S / count)) would leave roots unassigned, so such launches take the LPT map
    GatherArgs am = a;
    if (am.block_map == 0 && (am.split & 7) != 0) am.block_map = 3;
    if (a.wait_ev) {  // another context's tile kernel first (bre_set_gather_after)
        const hipError_t ew = hipStreamWaitEvent(s, a.wait_ev, 0);
        if (ew != hipSuccess) return ew;
    }
    if (a.user_start) {  // the caller's timing: the tile kernel alone (bre_set_gather_events)
        const hipError_t es = hipEventRecord(a.user_start, s);
        if (es != hipSuccess) return es;
    }
#define BRE_LAUNCH_TILE(C, W)                                                                                    \
    hipLaunchKernelGGL((k_gather_tile<C, W>), grid4, dim3(kTileBlock), 0, s, a.nseg, a.o, a.p, a.d, a.tmax,      \
                       a.segrec, a.R, a.partial, pcnt, a.recs, a.pow, a.bset, a.nodes, a.nodes4, a.nvalid,        \
                       a.leaf_size,                                                                        \
                       a.roots, a.split, a.ctr, stack_cap, (int)a.prefilter, am.block_map, a.tscan, a.margin, tax)
    if (counters) {
        BRE_LAUNCH_TILE(true, 1);
    } else if (a.occupancy == 1) {
        BRE_LAUNCH_TILE(false, 1);
    } else if (a.occupancy == 4) {
        BRE_LAUNCH_TILE(false, 4);
    } else if (a.occupancy == 5) {
        BRE_LAUNCH_TILE(false, 5);
    } else if (a.occupancy == 6) {
        BRE_LAUNCH_TILE(false, 6);
    } else if (a.occupancy == 8) {
        BRE_LAUNCH_TILE(false, 8);
    } else {
        BRE_LAUNCH_TILE(false, 7);
    }
#undef BRE_LAUNCH_TILE
    hipError_t e4 = hipGetLastError();
    if (e4 != hipSuccess) return e4;
    if (a.done_ev) {
        e4 = hipEventRecord(a.done_ev, s);
        if (e4 != hipSuccess) return e4;
    }
    if (a.user_end) {
        e4 = hipEventRecord(a.user_end, s);
        if (e4 != hipSuccess) return e4;
    }
    hipLaunchKernelGGL(k_reduce, dim3((unsigned int)((a.nseg + kPassBlock - 1) / kPassBlock)), dim3(kPassBlock), 0, s, a.nseg, a.partial, pcnt,
                       a.roots, a.split, a.pixel, a.npix, a.accum, a.seg_rgb, a.seg_counts, a.seg_index, a.ctr);
    return hipGetLastError();
}

hipError_t launch_zero_outputs(const GatherArgs &a, hipStream_t s) {
    if (a.nseg == 0 || (!a.seg_rgb && !a.seg_counts)) return hipSuccess;
    hipLaunchKernelGGL(k_zero_seg, dim3((unsigned int)((a.nseg + 63) / 64)), dim3(64), 0, s, a.nseg, a.seg_rgb,
                       a.seg_counts, a.seg_index);
    return hipGetLastError();
}

}  // namespace bre

#if BRE_WAVE_TIMES
// study builds only: the last tile-kernel launch's per-block start and end times (zeros for blocks that
// exited at once), n blocks into out[0..n) and out[n..2n)
extern "C" int bre_study_wave_times(int64_t n, unsigned long long *out) {
    if (n > bre::kWaveTimes) n = bre::kWaveTimes;
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(bre::g_wave_t), (size_t)n * 8, 0, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    if (hipMemcpyFromSymbol(out + n, HIP_SYMBOL(bre::g_wave_t), (size_t)n * 8, (size_t)bre::kWaveTimes * 8,
                            hipMemcpyDeviceToHost) != hipSuccess)
        return 2;
    return 0;
}
#endif

