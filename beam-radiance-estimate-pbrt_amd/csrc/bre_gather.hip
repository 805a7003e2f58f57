// bre_gather.hip — the beam-radiance gather on gfx950.
//
// One launch replaces the reference's per-segment loop body (photonbeam.cpp:494-508) for every
// camera segment of an iteration: PhotonBeamBVH::Intersect (photonbeambvh.cpp:685-723) becomes a
// traversal of the GPU BVH, and each beam reached is re-tested with the reference's own slab test
// on its own (group) box, so the candidate set is the reference's exactly; each candidate then
// runs ComputeClosestPoints and the 1D kernel 1e-5*powerEnd*sqrt(1-(d/(R+r))^2) in the
// reference's float arithmetic (bre_math.h).
//
// Kernel 1 (k_gather_wave, default): wave-packet traversal.  A wave owns 64 segments (lanes);
// the traversal stack and the current node are wave-uniform, so node and beam records are read
// with scalar (SMEM) loads once per wave and broadcast to all lanes through SGPRs; the descent
// decision is a 64-lane ballot.  Coherent segments (neighbouring pixels) share almost all
// candidates, so one 64-B beam line feeds 64 closest-point evaluations.
// Kernel 2 (k_gather_thread): classic thread-per-segment traversal with a per-thread stack in
// LDS, for incoherent segment sets.
#include <hip/hip_runtime.h>

#include <float.h>

#include "bre_device.h"
#include "bre_math.h"

namespace bre {

namespace {

constexpr int kWaveBlock = 256;    // 4 waves
constexpr int kThreadBlock = 128;  // 2 waves, 32 KiB LDS stack


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
};
__device__ __forceinline__ BeamV load_beam(const BeamRec *__restrict__ recs, int64_t i) {
    const float4 *q = reinterpret_cast<const float4 *>(recs + i);
    const float4 x = q[0], y = q[1], z = q[2], w = q[3];
    BeamV r;
    r.box = Box6{x.x, x.y, x.z, x.w, y.x, y.y};
    r.b0 = mk(y.z, y.w, z.x);
    r.bu = mk(z.y, z.z, z.w);
    r.mag_b = w.x;
    r.radius = w.y;
    return r;
}

struct Lane {
    f3 o, p, au;
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
        L.o = L.p = L.au = L.inv = L.invs = mk(0.f, 0.f, 0.f);
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
    L.tmax = tmax[s];
    // invDir(1 / ray.d.x, ...), dirIsNeg = invDir < 0  (photonbeambvh.cpp:690-691)
    L.inv = mk(1 / dd.x, 1 / dd.y, 1 / dd.z);
    L.invs = mk(sanitize_inv(L.inv.x), sanitize_inv(L.inv.y), sanitize_inv(L.inv.z));
    L.has_inf = isinf(L.inv.x) | isinf(L.inv.y) | isinf(L.inv.z);
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

// Evaluate one beam record for one lane: reference box test, closest points, kernel.
struct Prof {
    unsigned long long leaves = 0, beams = 0, ccp_waves = 0, rejects = 0, useful = 0;
};

template <bool COUNT, bool PREF>
__device__ __forceinline__ void eval_beam(const Lane &L, bool lane_on, const BeamV &r, const float4 *__restrict__ pw,
                                          int64_t bi, float R, float &cr, float &cg, float &cb, int &cand,
                                          int &contrib, Prof &pf, int dbg = 0) {
    // candidate: the reference's own slab test on the beam's (group) box.  For a lane whose 1/d has
    // no infinite component, node_test(box, inv) is the same decision (bre_math.h); lanes with an
    // axis-parallel direction (inf, possible NaN paths) take the literal statement.
    float te;
    bool hit = lane_on & node_test(r.box, L.o, L.invs, L.tmax, te);
    if (__ballot(L.has_inf) != 0ull) {
        if (L.has_inf) hit = lane_on & slab_test(r.box, L.o, L.inv, L.n0, L.n1, L.n2, L.tmax, nullptr);
    }
    if (COUNT) cand += hit;
    if (__ballot(hit) == 0ull) return;  // wave-uniform
    if (COUNT) ++pf.useful;
    if (dbg == 2) return;  // timing-only: candidate tests, no distance work
    const float maxd = R + r.radius;    // MaxDistance = currentBeamRadius + beam->radius
    bool need = hit;
    if (PREF) {
        need = hit & !far_from_lines(L, r, maxd);
        if (COUNT) pf.rejects += hit & !need;
        if (__ballot(need) == 0ull) return;
    }
    if (dbg == 3) return;  // timing-only: no exact closest-point code
    if (COUNT) {
        const unsigned long long m = __ballot(need);
        if ((int)(threadIdx.x & 63) == __ffsll((long long)m) - 1) ++pf.ccp_waves;
    }
    if (need) {
        float dist;
        const bool ok = closest_distance(L.o, L.p, L.au, L.mag_a, r.b0, r.bu, r.mag_b, dist);
        if (ok & (dist < maxd)) {
            const float rr = dist / maxd;
            const float w = sqrtf(1.0f - rr * rr);
            const float4 pv = pw[bi];
            cr += pv.x * w;
            cg += pv.y * w;
            cb += pv.z * w;
            if (COUNT) ++contrib;
        }
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
                atomicOr(&ctr->flags, 2u);
            } else if (cr != 0.f || cg != 0.f || cb != 0.f) {
                atomicAdd(&accum[3 * (int64_t)px], cr);
                atomicAdd(&accum[3 * (int64_t)px + 1], cg);
                atomicAdd(&accum[3 * (int64_t)px + 2], cb);
            }
        }
        if (COUNT && seg_counts) {
            seg_counts[2 * s] = cand;
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

// Wave-packet traversal of one BVH subtree.  Grid = (segment groups of 256) x S subtrees with
// subtree = blockIdx % S: the S work roots partition the beams, so every (packet, subtree) pair is
// an independent work item (8x the waves of one full traversal per packet: load balance and latency
// hiding), and with S = 8 all blocks of one subtree are dealt to one XCD under the round-robin
// placement (L2 affinity; speed only, never correctness).  Per-subtree partial sums go to
// partial[sub][seg] and are summed in subtree order by k_reduce (deterministic results).
template <bool COUNT, bool PREF>
__global__ __launch_bounds__(kWaveBlock) void k_gather_wave(
    int64_t nseg, const float *__restrict__ so, const float *__restrict__ sp_, const float *__restrict__ sd,
    const float *__restrict__ stmax, float R, float *__restrict__ partial, int32_t *__restrict__ seg_counts,
    const BeamRec *__restrict__ recs, const float4 *__restrict__ pw, const Node *__restrict__ nodes, int64_t nvalid,
    int leaf_size, const int32_t *__restrict__ roots, int S, DevCounters *ctr, int dbg) {
    __shared__ int32_t stk[kWaveBlock / 64][kStackDepth];
    // Block -> (subtree, packet group).  Blocks b and b+8 share an XCD under the observed
    // round-robin dispatch, so for S >= 8 XCD (b & 7) is given the S/8 consecutive work roots
    // below one depth-3 node: each XCD's L2 serves one eighth of the tree (speed only).
    int sub;
    int64_t grp;
    if (S >= 8) {
        const unsigned per = (unsigned)S >> 3;
        const unsigned q = blockIdx.x >> 3;
        sub = (int)((blockIdx.x & 7u) * per + q % per);
        grp = q / per;
    } else {
        sub = (int)(blockIdx.x % (unsigned)S);
        grp = blockIdx.x / (unsigned)S;
    }
    if (sub >= roots[S]) return;  // fewer work roots than S (small trees): whole block exits
    const int w = threadIdx.x >> 6;
    const int64_t s = grp * kWaveBlock + threadIdx.x;
    Lane L;
    const bool valid = load_lane(s, nseg, so, sp_, sd, stmax, L);
    float cr = 0.f, cg = 0.f, cb = 0.f;
    int cand = 0, contrib = 0;
    unsigned long long visits = 0;
    Prof pf;

    if (__ballot(valid) != 0ull) {
        const int32_t root = roots[sub];
        if (root < 0) {
            // the work root is a leaf cluster: evaluate it directly
            const int64_t first = (int64_t)(~root) * leaf_size;
            const int cnt = (int)min((int64_t)leaf_size, nvalid - first);
            if (COUNT) {
                ++pf.leaves;
                pf.beams += cnt;
            }
            for (int j = 0; j < cnt; ++j)
                eval_beam<COUNT, PREF>(L, valid, load_beam(recs, first + j), pw, first + j, R, cr, cg, cb, cand,
                                       contrib, pf, dbg);
        } else {
            int node = root;
            int sp = 0;
            while (true) {
                node = __builtin_amdgcn_readfirstlane(node);
                const NodeV n = load_node(nodes, node);
                if (COUNT) ++visits;
                const int32_t c0 = n.c0, c1 = n.c1;
                float te0 = 0.f, te1 = 0.f;
                const bool h0 = valid & (c0 != kEmptyChild) & node_test(n.b0, L.o, L.invs, L.tmax, te0);
                const bool h1 = valid & (c1 != kEmptyChild) & node_test(n.b1, L.o, L.invs, L.tmax, te1);
                const unsigned long long m0 = __ballot(h0), m1 = __ballot(h1);
                // leaves are evaluated in place
                bool go0 = m0 != 0ull, go1 = m1 != 0ull;
                if (dbg == 1) {  // timing-only build: traversal without leaf work
                    if (go0 && c0 < 0) go0 = false;
                    if (go1 && c1 < 0) go1 = false;
                }
                if (go0 && c0 < 0) {
                    const int64_t first = (int64_t)(~c0) * leaf_size;
                    const int cnt = (int)min((int64_t)leaf_size, nvalid - first);
                    if (COUNT) {
                        ++pf.leaves;
                        pf.beams += cnt;
                    }
                    for (int j = 0; j < cnt; ++j)
                        eval_beam<COUNT, PREF>(L, h0, load_beam(recs, first + j), pw, first + j, R, cr, cg, cb, cand,
                                               contrib, pf, dbg);
                    go0 = false;
                }
                if (go1 && c1 < 0) {
                    const int64_t first = (int64_t)(~c1) * leaf_size;
                    const int cnt = (int)min((int64_t)leaf_size, nvalid - first);
                    if (COUNT) {
                        ++pf.leaves;
                        pf.beams += cnt;
                    }
                    for (int j = 0; j < cnt; ++j)
                        eval_beam<COUNT, PREF>(L, h1, load_beam(recs, first + j), pw, first + j, R, cr, cg, cb, cand,
                                               contrib, pf, dbg);
                    go1 = false;
                }
                if (go0 && go1) {
                    // near child first, judged by the first lane that enters both
                    const unsigned long long both = m0 & m1;
                    bool first0 = true;
                    if (both != 0ull) {
                        const int fl = __ffsll((long long)both) - 1;
                        const float a = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(te0), fl));
                        const float b = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(te1), fl));
                        first0 = !(b < a);
                    }
                    const int near = first0 ? c0 : c1, far = first0 ? c1 : c0;
                    if (sp >= kStackDepth) {
                        if ((threadIdx.x & 63) == 0) atomicOr(&ctr->flags, 1u);
                        break;
                    }
                    stk[w][sp] = far;  // every lane writes the same value
                    ++sp;
                    node = near;
                } else if (go0) {
                    node = c0;
                } else if (go1) {
                    node = c1;
                } else {
                    if (sp == 0) break;
                    --sp;
                    node = stk[w][sp];
                }
            }
        }
    }
    if (valid) {
        float *dst = partial + 3 * ((int64_t)sub * nseg + s);
        dst[0] = cr;
        dst[1] = cg;
        dst[2] = cb;
        if (COUNT && seg_counts) {
            atomicAdd(&seg_counts[2 * s], cand);
            atomicAdd(&seg_counts[2 * s + 1], contrib);
        }
    }
    if (COUNT) {
        unsigned long long c = valid ? (unsigned long long)cand : 0ull;
        unsigned long long k = valid ? (unsigned long long)contrib : 0ull;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            c += __shfl_xor(c, off);
            k += __shfl_xor(k, off);
        }
        unsigned long long rj = pf.rejects;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) rj += __shfl_xor(rj, off);
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(&ctr->candidates, c);
            atomicAdd(&ctr->contributions, k);
            atomicAdd(&ctr->node_visits, visits);
            atomicAdd(&ctr->leaf_visits, pf.leaves);
            atomicAdd(&ctr->beam_evals, pf.beams);
            atomicAdd(&ctr->useful_beam_evals, pf.useful);
            atomicAdd(&ctr->prefilter_rejects, rj);
        }
        // ccp_waves is counted by the first active lane of each execution: sum over lanes
        unsigned long long cw = pf.ccp_waves;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) cw += __shfl_xor(cw, off);
        if ((threadIdx.x & 63) == 0) atomicAdd(&ctr->ccp_wave_evals, cw);
    }
}

// Sum the per-subtree partials of each segment in subtree order; write seg_rgb and add the
// segment's sum to its pixel (one float atomic per channel, PhotonBeamPixel::Ld +=).
__global__ __launch_bounds__(256) void k_reduce(int64_t nseg, const float *__restrict__ partial,
                                                const int32_t *__restrict__ roots, int S,
                                                const int32_t *__restrict__ pixel, int64_t npix,
                                                float *__restrict__ accum, float *__restrict__ seg_rgb,
                                                DevCounters *ctr) {
    const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= nseg) return;
    const int nr = roots[S];
    float cr = 0.f, cg = 0.f, cb = 0.f;
    for (int k = 0; k < nr; ++k) {
        const float *q = partial + 3 * ((int64_t)k * nseg + s);
        cr += q[0];
        cg += q[1];
        cb += q[2];
    }
    if (seg_rgb) {
        seg_rgb[3 * s] = cr;
        seg_rgb[3 * s + 1] = cg;
        seg_rgb[3 * s + 2] = cb;
    }
    if (accum) {
        const int32_t px = pixel[s];
        if (px < 0 || px >= npix) {
            atomicOr(&ctr->flags, 2u);
        } else if (cr != 0.f || cg != 0.f || cb != 0.f) {
            atomicAdd(&accum[3 * (int64_t)px], cr);
            atomicAdd(&accum[3 * (int64_t)px + 1], cg);
            atomicAdd(&accum[3 * (int64_t)px + 2], cb);
        }
    }
}

// Work roots: the BVH frontier at depth log2(S) (leaves above it stay in the frontier).
__global__ void k_roots(const Node *__restrict__ nodes, int S, int32_t *__restrict__ roots) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int32_t cur[kMaxSplit], nxt[kMaxSplit];
    int n = 1;
    cur[0] = 0;
    while (true) {
        int m = 0;
        bool fits = true;
        for (int i = 0; i < n; ++i) m += (cur[i] >= 0) ? 2 : 1;
        if (m > S) fits = false;
        bool grew = false;
        if (fits) {
            m = 0;
            for (int i = 0; i < n; ++i) {
                if (cur[i] >= 0) {
                    const Node &nd = nodes[cur[i]];
                    if (nd.child[0] != kEmptyChild) nxt[m++] = nd.child[0];
                    if (nd.child[1] != kEmptyChild) nxt[m++] = nd.child[1];
                    grew = true;
                } else {
                    nxt[m++] = cur[i];
                }
            }
        }
        if (!fits || !grew) break;
        for (int i = 0; i < m; ++i) cur[i] = nxt[i];
        n = m;
    }
    for (int i = 0; i < n; ++i) roots[i] = cur[i];
    for (int i = n; i < S; ++i) roots[i] = kEmptyChild;
    roots[S] = n;
}

template <bool COUNT>
__global__ __launch_bounds__(kThreadBlock) void k_gather_thread(
    int64_t nseg, const float *__restrict__ so, const float *__restrict__ sp_, const float *__restrict__ sd,
    const float *__restrict__ stmax, const int32_t *__restrict__ pixel, float R, int64_t npix,
    float *__restrict__ accum, float *__restrict__ seg_rgb, int32_t *__restrict__ seg_counts,
    const BeamRec *__restrict__ recs, const float4 *__restrict__ pw, const Node *__restrict__ nodes, int64_t nvalid,
    int leaf_size, DevCounters *ctr) {
    __shared__ int32_t stk[kThreadStackDepth][kThreadBlock];
    const int tid = threadIdx.x;
    const int64_t s = (int64_t)blockIdx.x * kThreadBlock + tid;
    Lane L;
    const bool valid = load_lane(s, nseg, so, sp_, sd, stmax, L);
    float cr = 0.f, cg = 0.f, cb = 0.f;
    int cand = 0, contrib = 0;
    unsigned long long visits = 0;
    Prof pf;
    if (valid && nvalid > 0) {
        int node = 0;
        int sp = 0;
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
                    eval_beam<COUNT, false>(L, true, load_beam(recs, first + j), pw, first + j, R, cr, cg, cb, cand, contrib, pf);
                h0 = false;
            }
            if (h1 && c1 < 0) {
                const int64_t first = (int64_t)(~c1) * leaf_size;
                const int cnt = (int)min((int64_t)leaf_size, nvalid - first);
                for (int j = 0; j < cnt; ++j)
                    eval_beam<COUNT, false>(L, true, load_beam(recs, first + j), pw, first + j, R, cr, cg, cb, cand, contrib, pf);
                h1 = false;
            }
            if (h0 && h1) {
                const bool first0 = !(te1 < te0);
                if (sp >= kThreadStackDepth) {
                    atomicOr(&ctr->flags, 1u);
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

__global__ void k_zero_seg(int64_t nseg, float *__restrict__ seg_rgb, int32_t *__restrict__ seg_counts) {
    const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= nseg) return;
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

hipError_t launch_roots(const Node *nodes, int S, int32_t *roots, hipStream_t s) {
    hipLaunchKernelGGL(k_roots, dim3(1), dim3(64), 0, s, nodes, S, roots);
    return hipGetLastError();
}

hipError_t launch_gather(const GatherArgs &a, int kernel, bool counters, hipStream_t s) {
    if (a.nseg == 0) return hipSuccess;
    if (kernel == 2) {
        const dim3 grid((unsigned int)((a.nseg + kThreadBlock - 1) / kThreadBlock));
        if (counters)
            hipLaunchKernelGGL(k_gather_thread<true>, grid, dim3(kThreadBlock), 0, s, a.nseg, a.o, a.p, a.d, a.tmax,
                               a.pixel, a.R, a.npix, a.accum, a.seg_rgb, a.seg_counts, a.recs, a.pow, a.nodes,
                               a.nvalid, a.leaf_size, a.ctr);
        else
            hipLaunchKernelGGL(k_gather_thread<false>, grid, dim3(kThreadBlock), 0, s, a.nseg, a.o, a.p, a.d, a.tmax,
                               a.pixel, a.R, a.npix, a.accum, a.seg_rgb, a.seg_counts, a.recs, a.pow, a.nodes,
                               a.nvalid, a.leaf_size, a.ctr);
        return hipGetLastError();
    }
    if (counters && a.seg_counts) {
        hipError_t e = hipMemsetAsync(a.seg_counts, 0, sizeof(int32_t) * 2 * (size_t)a.nseg, s);
        if (e != hipSuccess) return e;
    }
    const int64_t groups = (a.nseg + kWaveBlock - 1) / kWaveBlock;
    const dim3 grid((unsigned int)(groups * a.split));
#define BRE_LAUNCH_WAVE(C, P)                                                                                   \
    hipLaunchKernelGGL((k_gather_wave<C, P>), grid, dim3(kWaveBlock), 0, s, a.nseg, a.o, a.p, a.d, a.tmax, a.R, \
                       a.partial, a.seg_counts, a.recs, a.pow, a.nodes, a.nvalid, a.leaf_size, a.roots, a.split,  \
                       a.ctr, a.debug_mode)
    if (counters) {
        if (a.prefilter) BRE_LAUNCH_WAVE(true, true);
        else BRE_LAUNCH_WAVE(true, false);
    } else {
        if (a.prefilter) BRE_LAUNCH_WAVE(false, true);
        else BRE_LAUNCH_WAVE(false, false);
    }
#undef BRE_LAUNCH_WAVE
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_reduce, dim3((unsigned int)((a.nseg + 255) / 256)), dim3(256), 0, s, a.nseg, a.partial,
                       a.roots, a.split, a.pixel, a.npix, a.accum, a.seg_rgb, a.ctr);
    return hipGetLastError();
}

hipError_t launch_zero_outputs(const GatherArgs &a, hipStream_t s) {
    if (a.nseg == 0 || (!a.seg_rgb && !a.seg_counts)) return hipSuccess;
    hipLaunchKernelGGL(k_zero_seg, dim3((unsigned int)((a.nseg + 255) / 256)), dim3(256), 0, s, a.nseg, a.seg_rgb,
                       a.seg_counts);
    return hipGetLastError();
}

}  // namespace bre
