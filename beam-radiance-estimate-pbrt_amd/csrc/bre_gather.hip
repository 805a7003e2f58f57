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
#include "bre_lane.h"
#include "bre_math.h"

namespace bre {

namespace {

constexpr int kWaveBlock = 256;    // 4 waves
constexpr int kThreadBlock = 128;  // 2 waves, 32 KiB LDS stack


// Evaluate one beam record for one lane: reference box test, closest points, kernel.
struct Prof {
    unsigned long long leaves = 0, beams = 0, ccp_waves = 0, rejects = 0, useful = 0;
};

template <bool COUNT, bool PREF, bool PWREG = false>
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
            float px, py, pz;
            if (PWREG) {
                px = r.pw.x;
                py = r.pw.y;
                pz = r.pw.z;
            } else {
                const float4 pv = pw[bi];
                px = pv.x;
                py = pv.y;
                pz = pv.z;
            }
            cr += px * w;
            cg += py * w;
            cb += pz * w;
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

// Depth-first wave-packet traversal of one work root (kernel 1, and kernel 3's path for loose
// packets): the current node and the stack are wave-uniform, node and beam lines are SMEM loads,
// each lane tests both children with node_test and the descent is a ballot.
template <bool COUNT, bool PREF>
__device__ __forceinline__ void dfs_packet(const Lane &L, bool valid, int32_t root, int32_t *stk,
                                           const BeamRec *__restrict__ recs, const float4 *__restrict__ pw,
                                           const Node *__restrict__ nodes, int64_t nvalid, int leaf_size, float R,
                                           float &cr, float &cg, float &cb, int &cand, int &contrib,
                                           unsigned long long &visits, Prof &pf, DevCounters *ctr, int dbg) {
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
                stk[sp] = far;  // every lane writes the same value
                ++sp;
                node = near;
            } else if (go0) {
                node = c0;
            } else if (go1) {
                node = c1;
            } else {
                if (sp == 0) break;
                --sp;
                node = stk[sp];
            }
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
    const float *__restrict__ stmax, float R, float *__restrict__ partial, int32_t *__restrict__ pcnt,
    const BeamRec *__restrict__ recs, const float4 *__restrict__ pw, const Node *__restrict__ nodes, int64_t nvalid,
    int leaf_size, const int32_t *__restrict__ roots, int S, DevCounters *ctr, int dbg,
    const uint8_t *__restrict__ redo) {
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
    // behind kernel 3, only the packets it handed over (incoherent, or out of LDS stack) run here
    if (redo) {  // per wave (one packet): a ragged last packet keeps all its lanes
        const int64_t pk = (grp * kWaveBlock + (int64_t)w * 64) >> 6;
        if (pk * 64 >= nseg || !redo[pk]) return;
    }
    Lane L;
    const bool valid = load_lane(s, nseg, so, sp_, sd, stmax, L);
    float cr = 0.f, cg = 0.f, cb = 0.f;
    int cand = 0, contrib = 0;
    unsigned long long visits = 0;
    Prof pf;

    if (__ballot(valid) != 0ull) {
        dfs_packet<COUNT, PREF>(L, valid, roots[sub], stk[w], recs, pw, nodes, nvalid, leaf_size, R, cr, cg, cb, cand,
                                contrib, visits, pf, ctr, dbg);
    }
    if (valid) {
        float *dst = partial + 3 * ((int64_t)sub * nseg + s);
        dst[0] = cr;
        dst[1] = cg;
        dst[2] = cb;
        if (COUNT) {
            pcnt[2 * ((int64_t)sub * nseg + s)] = cand;
            pcnt[2 * ((int64_t)sub * nseg + s) + 1] = contrib;
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
        (void)c;
        (void)k;
        if ((threadIdx.x & 63) == 0) {
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


// ---------------------------------------------------------------------------------------------
// Kernel 3 (k_gather_proxy): packet-proxy traversal.  A wave owns one packet of 64 coherent
// segments and one BVH work root.  Instead of walking the tree node by node with all 64 lanes
// testing the same node (kernel 1), each lane takes a DIFFERENT node from a wave-shared LDS stack
// and tests its two children against a conservative proxy of the whole packet (interval slab test
// over the packet's origin box x inverse-direction box, plus the packet's segment AABB): 64 nodes
// per step, one vector load per lane, no dependent per-node latency.  Hit leaves append their beams
// to an LDS candidate list; every 64 candidates are loaded with one vector load per lane and
// broadcast one by one (v_readlane) to all lanes, which run the exact reference tests per lane.
//
// Conservativeness chain (why no candidate is lost): a lane's exact slab hit on a beam box =>
// node_test on that box (bre_math.h) => node_test on every ancestor (monotone under containment)
// => proxy_test on every ancestor (the lane's float values (b - o)*v lie between the corner values
// the proxy computes with the same float operations, because rounding is monotone and the
// function is bilinear).  The proxy only decides WHICH beams get the exact per-lane test.
constexpr int kProxyStack = 1024;  // LDS node-stack entries per wave (>= kStackDepth: reused by dfs); 550 seen at C2
constexpr float kLooseCos = 0.9976f;  // default: packets whose directions spread > ~4 deg use the dfs path
constexpr int kProxyMaxLeaf = 4;             // kernel 3 needs leaf clusters of <= 4 beams
constexpr int kCandCap = 64 + 2 * 64 * kProxyMaxLeaf;  // leftover + one step's leaf beams

struct Proxy {
    float olo[3], ohi[3];   // packet origin box
    float ilo[3], ihi[3];   // packet box of sanitised 1/d
    int sgn[3];             // +1 / -1 if every lane's 1/d_i has that sign, 0 if mixed
    float alo[3], ahi[3];   // AABB of all segments [o, o + tmax*d], padded
    float tmax;             // max ray.tMax
};

__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = fminf(v, __shfl_xor(v, off));
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
    return v;
}

__device__ __forceinline__ Proxy make_proxy(const Lane &L, bool valid) {
    Proxy P;
    const float o[3] = {L.o.x, L.o.y, L.o.z};
    const float iv[3] = {L.invs.x, L.invs.y, L.invs.z};
    const float dd[3] = {L.d.x, L.d.y, L.d.z};
    float mag = 0.f;
#pragma unroll
    for (int k = 0; k < 3; ++k) mag = fmaxf(mag, fabsf(o[k]) + L.tmax * fabsf(dd[k]));
    const float pad = 1e-5f * mag + 1e-6f;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float e = o[k] + L.tmax * dd[k];
        P.olo[k] = wave_min(valid ? o[k] : FLT_MAX);
        P.ohi[k] = wave_max(valid ? o[k] : -FLT_MAX);
        P.ilo[k] = wave_min(valid ? iv[k] : FLT_MAX);
        P.ihi[k] = wave_max(valid ? iv[k] : -FLT_MAX);
        P.alo[k] = wave_min(valid ? fminf(o[k], e) - pad : FLT_MAX);
        P.ahi[k] = wave_max(valid ? fmaxf(o[k], e) + pad : -FLT_MAX);
        P.sgn[k] = (P.ilo[k] > 0.f) ? 1 : ((P.ihi[k] < 0.f) ? -1 : 0);
    }
    P.tmax = wave_max(valid ? L.tmax : -FLT_MAX);
    return P;
}

// Packet bundle for kernel 3's packet-level line-distance reject.  A line C (point co, unit
// direction cu) and delta >= the distance of every valid lane's segment END POINTS from C.  The
// distance to a line is convex along a segment, so every point of every lane's segment lies within
// delta of C, and for any beam line B: dist(segment_i, B) >= dist(C, B) - delta.  One lane-wide
// evaluation per beam (64 beams at once) then rejects a beam for all 64 segments, before the
// per-lane prefilter.  delta and the coordinate bound are inflated for rounding.
struct Bundle {
    f3 co, cu;
    float delta;  // FLT_MAX disables the test
    float omax;   // max over valid lanes of Lane::omax (bounds every segment-side coordinate)
};

template <int G>
__device__ __forceinline__ float grp_sum(float v) {
#pragma unroll
    for (int off = G / 2; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}
template <int G>
__device__ __forceinline__ float grp_max(float v) {
#pragma unroll
    for (int off = G / 2; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
    return v;
}

// The bundle of the valid lanes of each aligned group of G lanes (G = 64: the whole packet); every
// lane returns its own group's bundle.  All lanes must call (shuffles stay inside a group).
template <int G>
__device__ __forceinline__ Bundle make_bundle_g(const Lane &L, bool valid) {
    const int lane = threadIdx.x & 63;
    const unsigned long long m = __ballot(valid);
    const unsigned long long gm = G == 64 ? m : ((m >> (lane & ~(G - 1))) & ((1ull << G) - 1ull));
    const int cnt = __popcll(gm);
    const float n = (float)(cnt > 0 ? cnt : 1);
    Bundle K;
    K.co = mk(grp_sum<G>(valid ? L.o.x : 0.f) / n, grp_sum<G>(valid ? L.o.y : 0.f) / n,
              grp_sum<G>(valid ? L.o.z : 0.f) / n);
    const f3 su = mk(grp_sum<G>(valid ? L.au.x : 0.f), grp_sum<G>(valid ? L.au.y : 0.f), grp_sum<G>(valid ? L.au.z : 0.f));
    const float sl = sqrtf(lensq3(su));
    K.omax = grp_max<G>(valid ? L.omax : 0.f);
    const bool ok = cnt > 0 && sl > 0.f && isfinite(sl);
    K.cu = ok ? mk(su.x / sl, su.y / sl, su.z / sl) : mk(0.f, 0.f, 1.f);
    const auto perp = [&](f3 x) {
        const f3 t = sub3(x, K.co);
        const f3 c = mk(t.y * K.cu.z - t.z * K.cu.y, t.z * K.cu.x - t.x * K.cu.z, t.x * K.cu.y - t.y * K.cu.x);
        return sqrtf(lensq3(c));
    };
    const float dl = valid ? fmaxf(perp(L.o), perp(L.p)) : 0.f;
    const float cm = fmaxf(fmaxf(fabsf(K.co.x), fabsf(K.co.y)), fabsf(K.co.z));
    const float d = grp_max<G>(dl);
    K.delta = (ok && isfinite(d)) ? d * 1.0001f + 1e-5f * (K.omax + cm) + 1e-6f : FLT_MAX;
    return K;
}

__device__ __forceinline__ float uniform_f(float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); }

// The whole packet's bundle, wave-uniform: kept in SGPRs.
__device__ __forceinline__ Bundle make_bundle(const Lane &L, bool valid) {
    Bundle K = make_bundle_g<64>(L, valid);
    K.co = mk(uniform_f(K.co.x), uniform_f(K.co.y), uniform_f(K.co.z));
    K.cu = mk(uniform_f(K.cu.x), uniform_f(K.cu.y), uniform_f(K.cu.z));
    K.delta = uniform_f(K.delta);
    K.omax = uniform_f(K.omax);
    return K;
}

// far_from_lines_fast's bound for the bundle's line against a beam line, with maxd + delta: a
// rejection proves that every lane's computed ComputeClosestPoints distance is >= maxd.
__device__ __forceinline__ bool bundle_far(const Bundle &K, f3 b0, f3 bu, float maxd) {
    if (!(K.delta < 1e30f)) return false;
    const f3 t = sub3(b0, K.co);
    const f3 n = mk(__builtin_fmaf(K.cu.y, bu.z, -(K.cu.z * bu.y)), __builtin_fmaf(K.cu.z, bu.x, -(K.cu.x * bu.z)),
                    __builtin_fmaf(K.cu.x, bu.y, -(K.cu.y * bu.x)));
    const float nn = __builtin_fmaf(n.x, n.x, __builtin_fmaf(n.y, n.y, n.z * n.z));
    if (!(nn >= 1e-2f)) return false;
    const float tn = fabsf(__builtin_fmaf(t.x, n.x, __builtin_fmaf(t.y, n.y, t.z * n.z)));
    const float tl = fabsf(t.x) + fabsf(t.y) + fabsf(t.z);
    const float bmax = fmaxf(fmaxf(fabsf(b0.x), fabsf(b0.y)), fabsf(b0.z));
    const float mag = K.omax + bmax + 10.0f * tl + maxd + 1.0f;
    const float eps = 1e-5f * mag + 1e-6f;
    const float nl = __builtin_amdgcn_sqrtf(nn) * 1.000001f;
    return (tn - 1e-6f * tl) > ((maxd + K.delta) * 1.0001f + 2.0f * eps) * (nl + 1e-6f);
}

__device__ __forceinline__ float min4(float a, float b, float c, float d) { return fminf(fminf(a, b), fminf(c, d)); }
__device__ __forceinline__ float max4(float a, float b, float c, float d) { return fmaxf(fmaxf(a, b), fmaxf(c, d)); }

__device__ __forceinline__ bool proxy_test(const Proxy &P, const Box6 &b) {
    const float lo[3] = {b.lx, b.ly, b.lz}, hi[3] = {b.hx, b.hy, b.hz};
    bool ok = true;
    float tn = -FLT_MAX, tf = FLT_MAX;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        ok = ok & (hi[k] >= P.alo[k]) & (lo[k] <= P.ahi[k]);
        if (P.sgn[k] != 0) {  // wave-uniform
            const float bn = P.sgn[k] > 0 ? lo[k] : hi[k];
            const float bf = P.sgn[k] > 0 ? hi[k] : lo[k];
            const float n0 = bn - P.olo[k], n1 = bn - P.ohi[k];
            const float f0 = bf - P.olo[k], f1 = bf - P.ohi[k];
            tn = fmaxf(tn, min4(n0 * P.ilo[k], n0 * P.ihi[k], n1 * P.ilo[k], n1 * P.ihi[k]));
            tf = fminf(tf, max4(f0 * P.ilo[k], f0 * P.ihi[k], f1 * P.ilo[k], f1 * P.ihi[k]));
        }
    }
    tf = tf * slab_pad();
    return ok & (tn <= tf) & (tn < P.tmax) & (tf > 0.f);
}

// exclusive prefix sum of a small non-negative int over the wave
__device__ __forceinline__ int wave_excl_scan(int v, int &total) {
    const int lane = threadIdx.x & 63;
    int x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    total = __shfl(x, 63);
    return x - v;
}

template <bool COUNT, bool PREF>
__device__ __forceinline__ void proxy_batch(const Lane &L, bool valid, const int32_t *cand, int nb,
                                            const BeamRec *__restrict__ recs, const float4 *__restrict__ pw,
                                            float R, float &cr, float &cg, float &cb, int &ccount, int &contrib,
                                            Prof &pf, int dbg) {
    const int lane = threadIdx.x & 63;
    int bi = 0;
    BeamV mine;
    float4 mpw = make_float4(0.f, 0.f, 0.f, 0.f);
    if (lane < nb) {
        bi = cand[lane];
        mine = load_beam(recs, bi);
        mpw = pw[bi];
    } else {
        mine = BeamV{};
    }
    if (COUNT) pf.beams += nb;
    for (int j = 0; j < nb; ++j) {
        BeamV r;
        const auto rl = [&](float v) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j)); };
        r.box = Box6{rl(mine.box.lx), rl(mine.box.ly), rl(mine.box.lz), rl(mine.box.hx), rl(mine.box.hy),
                     rl(mine.box.hz)};
        r.b0 = mk(rl(mine.b0.x), rl(mine.b0.y), rl(mine.b0.z));
        r.bu = mk(rl(mine.bu.x), rl(mine.bu.y), rl(mine.bu.z));
        r.mag_b = rl(mine.mag_b);
        r.radius = rl(mine.radius);
        r.pw = mk(rl(mpw.x), rl(mpw.y), rl(mpw.z));
        eval_beam<COUNT, PREF, true>(L, valid, r, pw, 0, R, cr, cg, cb, ccount, contrib, pf, dbg);
    }
}

// Compacted form of proxy_batch (the default).  The batch's beam lines and powers are staged in
// LDS once (one 64-B line + 16 B per lane).  Per lane and beam only the conservative line-distance
// prefilter runs (beam line broadcast from LDS); the (beam, lane) pairs it keeps (~1 in 8 at C2)
// go to a ring in LDS, and every 64 of them (and the batch's remainder) run the reference's box
// test on the beam's group box, ComputeClosestPoints and the kernel with all lanes busy, one pair
// per lane, beam data read back from the staged lines, adding into the segment's LDS accumulator.
// The contributing pairs are the same (a contribution needs both the box hit and d < R + r; the
// prefilter only drops pairs with d >= R + r), each pair's value is computed by the same
// arithmetic, and a segment's pairs are summed in candidate-list order as in proxy_batch.
__device__ __forceinline__ int lanes_below(unsigned long long m) {
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

constexpr int kPQueue = 128;  // >= 63 left over + 64 appended by one beam

struct ProxyQ {
    float4 bst[64][2];     // staged lines of the current batch: (b0, |B|), (unit dir, radius)
    int32_t gid[64];       // their beam indices (box and power are read from L2 by pq_exact)
    float acc[3][64];      // per-segment RGB
    int32_t cnt[64];       // per-segment contribution counts (counters only)
    uint16_t q[kPQueue];   // ring: staged slot | segment lane << 8
};

// all lanes call; lanes < n take pair (first + lane) of the ring
template <bool COUNT>
__device__ __forceinline__ void pq_exact(ProxyQ &q, const Lane &M, int first, int n, float R,
                                         const BeamRec *__restrict__ recs, const float4 *__restrict__ pw, Prof &pf) {
    const int lane = threadIdx.x & 63;
    const bool on = lane < n;
    const unsigned qv = q.q[(first + (on ? lane : 0)) & (kPQueue - 1)];
    const int j = (int)(qv & 0xffu), sl = (int)(qv >> 8);
    const f3 o = mk(__shfl(M.o.x, sl), __shfl(M.o.y, sl), __shfl(M.o.z, sl));
    const f3 p = mk(__shfl(M.p.x, sl), __shfl(M.p.y, sl), __shfl(M.p.z, sl));
    const f3 au = mk(__shfl(M.au.x, sl), __shfl(M.au.y, sl), __shfl(M.au.z, sl));
    const f3 invs = mk(__shfl(M.invs.x, sl), __shfl(M.invs.y, sl), __shfl(M.invs.z, sl));
    const float mag_a = __shfl(M.mag_a, sl);
    const float tmax = __shfl(M.tmax, sl);
    const bool inf = __shfl((int)M.has_inf, sl) != 0;
    const int32_t bi = q.gid[j];
    const BeamV r = load_beam(recs, bi);  // one 64-B line per lane, L2-resident
    const Box6 &box = r.box;
    if (COUNT && lane == 0) ++pf.ccp_waves;
    // the reference's candidate test on the beam's (group) box, as eval_beam
    float te;
    bool hit = on & node_test(box, o, invs, tmax, te);
    if (__ballot(on & inf) != 0ull) {
        // shuffle with every lane active: ds_bpermute reads 0 from a lane outside EXEC
        const f3 d = mk(__shfl(M.d.x, sl), __shfl(M.d.y, sl), __shfl(M.d.z, sl));
        if (on & inf) {
            const f3 inv = mk(1 / d.x, 1 / d.y, 1 / d.z);
            hit = slab_test(box, o, inv, inv.x < 0, inv.y < 0, inv.z < 0, tmax, nullptr);
        }
    }
    if (__ballot(hit) == 0ull) return;
    if (hit) {
        const float maxd = R + r.radius;  // MaxDistance = currentBeamRadius + beam->radius
        float dist;
        const bool ok = closest_distance(o, p, au, mag_a, r.b0, r.bu, r.mag_b, dist);
        if (ok & (dist < maxd)) {
            const float rr = dist / maxd;
            const float wt = sqrtf(1.0f - rr * rr);
            const float4 pv = pw[bi];
            atomicAdd(&q.acc[0][sl], pv.x * wt);
            atomicAdd(&q.acc[1][sl], pv.y * wt);
            atomicAdd(&q.acc[2][sl], pv.z * wt);
            if (COUNT) atomicAdd(&q.cnt[sl], 1);
        }
    }
}

template <bool COUNT, bool PREF>
__device__ __forceinline__ void proxy_batch_q(ProxyQ &q, const Lane &L, bool valid, const int32_t *cand, int nb,
                                              const BeamRec *__restrict__ recs, const float4 *__restrict__ pw,
                                              float R, int &ccount, Prof &pf, int dbg, const Bundle &K) {
    const int lane = threadIdx.x & 63;
    // stage the batch, lane j holding beam j; the packet-level bundle test (one beam per lane)
    // drops beams that are far from every segment of the packet.  Kept beams are compacted in
    // candidate order (COUNT: all are staged, dropped ones flagged by ~index, because the
    // reference's candidate count needs every box test).
    int32_t bi = 0;
    float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0;
    bool keep = false;
    if (lane < nb) {
        bi = cand[lane];
        const float4 *src = reinterpret_cast<const float4 *>(recs + bi);
        const float4 b = src[1], c = src[2], d = src[3];
        s0 = make_float4(b.z, b.w, c.x, d.x);  // b0, |B|
        s1 = make_float4(c.y, c.z, c.w, d.y);  // unit dir, radius
        keep = !(PREF && bundle_far(K, mk(s0.x, s0.y, s0.z), mk(s1.x, s1.y, s1.z), R + s1.w));
    }
    int nk;
    if (COUNT) {
        if (lane < nb) {
            q.bst[lane][0] = s0;
            q.bst[lane][1] = s1;
            q.gid[lane] = keep ? bi : ~bi;
        }
        nk = nb;
    } else {
        const unsigned long long km = __ballot(keep);
        if (keep) {
            const int pos = lanes_below(km);
            q.bst[pos][0] = s0;
            q.bst[pos][1] = s1;
            q.gid[pos] = bi;
        }
        nk = __popcll(km);
    }
    if (COUNT) {
        pf.beams += nb;
        pf.useful += __popcll(__ballot(keep));  // beams kept by the bundle test
    }
    __builtin_amdgcn_wave_barrier();
    int qh = 0, qt = 0;  // wave-uniform ring head / tail (the ring is drained per batch)
    for (int j = 0; j < nk; ++j) {
        const float4 y = q.bst[j][0], z = q.bst[j][1];
        const f3 b0 = mk(y.x, y.y, y.z), bu = mk(z.x, z.y, z.z);
        bool need = valid;
        if (COUNT) need = need && q.gid[j] >= 0;
        if (PREF) need = need && !far_from_lines_fast(L.o, L.au, L.mag_a, L.omax, b0, bu, R + z.w);
        if (COUNT) {
            // the reference's candidate count C (box hits), for the parity tests
            const int32_t g = q.gid[j];
            const Box6 box = load_beam(recs, g >= 0 ? g : ~g).box;
            float te;
            bool hit = valid & node_test(box, L.o, L.invs, L.tmax, te);
            if (L.has_inf) hit = valid & slab_test(box, L.o, L.inv, L.n0, L.n1, L.n2, L.tmax, nullptr);
            ccount += hit;
            pf.rejects += hit & !need;
        }
        const unsigned long long m = __ballot(need);
        if (m == 0ull) continue;
        if (need) q.q[(qt + lanes_below(m)) & (kPQueue - 1)] = (uint16_t)(j | (lane << 8));
        qt += __popcll(m);
        __builtin_amdgcn_wave_barrier();
        if (qt - qh >= 64) {
            if (dbg != 2) pq_exact<COUNT>(q, L, qh, 64, R, recs, pw, pf);
            qh += 64;
            __builtin_amdgcn_wave_barrier();
        }
    }
    if (qt > qh && dbg != 2) pq_exact<COUNT>(q, L, qh, qt - qh, R, recs, pw, pf);
    __builtin_amdgcn_wave_barrier();
}

template <bool COUNT, bool PREF, int MINW>
__global__ __launch_bounds__(64, MINW) void k_gather_proxy(
    int64_t nseg, const float *__restrict__ so, const float *__restrict__ sp_, const float *__restrict__ sd,
    const float *__restrict__ stmax, float R, float *__restrict__ partial, int32_t *__restrict__ pcnt,
    const BeamRec *__restrict__ recs, const float4 *__restrict__ pw, const Node *__restrict__ nodes, int64_t nvalid,
    int leaf_size, const int32_t *__restrict__ roots, int S, DevCounters *ctr, int stack_limit, int dbg,
    uint8_t *__restrict__ redo, float loose_cos) {
    __shared__ int32_t stk[kProxyStack];
    __shared__ int32_t cand[kCandCap];
    __shared__ ProxyQ pq;
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
    if (sub >= roots[S]) return;
    const int lane = threadIdx.x & 63;
    const int64_t s = grp * 64 + lane;
    Lane L;
    const bool valid = load_lane(s, nseg, so, sp_, sd, stmax, L);
    float cr = 0.f, cg = 0.f, cb = 0.f;
    int ccount = 0, contrib = 0;
    Prof pf;
    unsigned long long tests = 0;
    int maxsp = 0;
    bool overflow = false;
    pq.acc[0][lane] = 0.f;
    pq.acc[1][lane] = 0.f;
    pq.acc[2][lane] = 0.f;
    pq.cnt[lane] = 0;

    // Incoherent packets (directions spread wider than kLooseCos) make the proxy useless: they take
    // the depth-first per-lane path instead (kernel 1's traversal, same exact per-lane tests).
    bool loose = false;
    if (__ballot(valid) != 0ull) {
        float sx = valid ? L.d.x : 0.f, sy = valid ? L.d.y : 0.f, sz = valid ? L.d.z : 0.f;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            sx += __shfl_xor(sx, off);
            sy += __shfl_xor(sy, off);
            sz += __shfl_xor(sz, off);
        }
        const float sn = sqrtf(sx * sx + sy * sy + sz * sz);
        const float dn = sqrtf(lensq3(L.d));
        const float c = (valid && sn > 0.f && dn > 0.f) ? (sx * L.d.x + sy * L.d.y + sz * L.d.z) / (sn * dn) : 1.0f;
        loose = wave_min(c) < loose_cos;
    }
    if (loose) {
        // handed to kernel 1 (depth-first per-lane traversal), which runs behind this launch
    } else if (__ballot(valid) != 0ull) {
        const Proxy P = make_proxy(L, valid);
        const Bundle K = make_bundle(L, valid);
        const int32_t root = roots[sub];
        int sp = 0, nc = 0;
        if (root < 0) {
            const int64_t first = (int64_t)(~root) * leaf_size;
            const int cnt = (int)min((int64_t)leaf_size, nvalid - first);
            if (lane < cnt) cand[lane] = (int32_t)(first + lane);
            nc = cnt;
        } else {
            if (lane == 0) stk[0] = root;
            sp = 1;
        }
        __builtin_amdgcn_wave_barrier();
        while (sp > 0 || nc > 0) {
            // 1. pop up to 64 nodes and issue their loads ...
            int n = 0;
            NodeV nd{};
            if (sp > 0) {
                n = min(64, sp);
                if (sp + n > stack_limit) n = stack_limit - sp;
                if (n <= 0) {
                    overflow = true;
                    break;
                }
                const int base = sp - n;
                int32_t node = 0;
                if (lane < n) node = stk[base + lane];
                __builtin_amdgcn_wave_barrier();
                sp = base;
                if (lane < n) nd = load_node(nodes, node);
            }
            // 2. ... and evaluate the full candidate batches gathered so far while they are in flight
            while (nc >= 64) {
                nc -= 64;
                if (dbg != 1)  // dbg 1: timing-only traversal
                    proxy_batch_q<COUNT, PREF>(pq, L, valid, cand + nc, 64, recs, pw, R, ccount, pf, dbg, K);
                __builtin_amdgcn_wave_barrier();
            }
            // 3. test the popped nodes' children against the packet proxy
            if (n > 0) {
                bool h0 = false, h1 = false;
                int32_t c0 = kEmptyChild, c1 = kEmptyChild;
                if (lane < n) {
                    c0 = nd.c0;
                    c1 = nd.c1;
                    h0 = (c0 != kEmptyChild) && proxy_test(P, nd.b0);
                    h1 = (c1 != kEmptyChild) && proxy_test(P, nd.b1);
                }
                if (COUNT) tests += n;
                // push interior children
                const bool p0 = h0 && c0 >= 0, p1 = h1 && c1 >= 0;
                int tot;
                const int pos = wave_excl_scan((int)p0 + (int)p1, tot);
                if (p0) stk[sp + pos] = c0;
                if (p1) stk[sp + pos + (int)p0] = c1;
                sp += tot;
                // append leaf beams
                int k0 = 0, k1 = 0;
                int64_t f0 = 0, f1 = 0;
                if (h0 && c0 < 0) {
                    f0 = (int64_t)(~c0) * leaf_size;
                    k0 = (int)min((int64_t)leaf_size, nvalid - f0);
                }
                if (h1 && c1 < 0) {
                    f1 = (int64_t)(~c1) * leaf_size;
                    k1 = (int)min((int64_t)leaf_size, nvalid - f1);
                }
                int ltot;
                const int lpos = wave_excl_scan(k0 + k1, ltot);
                for (int j = 0; j < k0; ++j) cand[nc + lpos + j] = (int32_t)(f0 + j);
                for (int j = 0; j < k1; ++j) cand[nc + lpos + k0 + j] = (int32_t)(f1 + j);
                nc += ltot;
                if (COUNT) {
                    pf.leaves += __popcll(__ballot(k0 > 0)) + __popcll(__ballot(k1 > 0));
                    maxsp = max(maxsp, sp);
                }
                __builtin_amdgcn_wave_barrier();
            }
            // 4. the stack is empty: evaluate what is left
            if (sp == 0) {
                while (nc > 0) {
                    const int nb = min(64, nc);
                    nc -= nb;
                    if (dbg != 1)
                        proxy_batch_q<COUNT, PREF>(pq, L, valid, cand + nc, nb, recs, pw, R, ccount, pf, dbg, K);
                    __builtin_amdgcn_wave_barrier();
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        cr = pq.acc[0][lane];
        cg = pq.acc[1][lane];
        cb = pq.acc[2][lane];
        contrib = pq.cnt[lane];
    }
    if (loose || overflow) {
        // kernel 1 redoes this packet for every subtree; nothing of this wave is kept
        if (lane == 0) {
            redo[grp] = 1;
            if (COUNT) atomicAdd(&ctr->redo_items, 1ull);
        }
        return;
    }
    if (valid) {
        float *dst = partial + 3 * ((int64_t)sub * nseg + s);
        dst[0] = cr;
        dst[1] = cg;
        dst[2] = cb;
        if (COUNT) {
            pcnt[2 * ((int64_t)sub * nseg + s)] = ccount;
            pcnt[2 * ((int64_t)sub * nseg + s) + 1] = contrib;
        }
    }
    if (COUNT) {
        unsigned long long c = valid ? (unsigned long long)ccount : 0ull;
        unsigned long long k = valid ? (unsigned long long)contrib : 0ull;
        unsigned long long rj = pf.rejects, cw = pf.ccp_waves;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            c += __shfl_xor(c, off);
            k += __shfl_xor(k, off);
            rj += __shfl_xor(rj, off);
            cw += __shfl_xor(cw, off);
        }
        (void)c;
        (void)k;
        if (lane == 0) {
            atomicAdd(&ctr->node_visits, tests);
            atomicAdd(&ctr->leaf_visits, pf.leaves);
            atomicAdd(&ctr->beam_evals, pf.beams);
            atomicAdd(&ctr->useful_beam_evals, pf.useful);
            atomicAdd(&ctr->prefilter_rejects, rj);
            atomicAdd(&ctr->ccp_wave_evals, cw);
            atomicMax(&ctr->max_stack, (unsigned int)maxsp);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Kernel 4 (k_gather_tile): wave-packet traversal over leaf TILES of up to 64 beams with two
// levels of wavefront compaction of the per-pair work.
//
// At dense candidate sets (the C2 Cornell fog: a camera segment passes ~16% of all beam boxes,
// and packets of incoherent bounce segments share few of them) the exact per-pair code executed
// under a 64-lane mask is the cost: a wave runs ComputeClosestPoints whenever ANY lane needs it,
// with ~3% of the lanes active.  Here:
//   1. a hit leaf tile's beam boxes are staged in LDS by one vector load per lane, and the tile is
//      scanned beam by beam with only the reference's box test per lane (~25 VALU ops, box read
//      by an LDS broadcast);
//   2. (segment lane, beam) pairs that pass are appended to a per-wave LDS queue (ballot +
//      mbcnt); every 64 queued pairs run the conservative distance prefilter with all lanes busy
//      (each lane takes one pair, its segment from LDS and the beam line from L2);
//   3. the prefilter's survivors go to a second queue; every 64 of those run
//      ComputeClosestPoints and the kernel, again one pair per lane, and add the contribution to
//      the segment's LDS accumulator.
// Same per-pair arithmetic as kernel 1; only the float summation order of a segment's
// contributions differs (deterministic: queue order is fixed by the traversal).
// Kernel 4's per-lane prefilter in separable form.  With t = b0 - o and n = au x bu,
//   t.n = au.(bu x b0) - bu.(o x au) = au.m0 - bu.q,
// so per (lane, beam) only two dot products and c = au.bu remain: m0 is staged per beam, q per lane.
// |n|^2 = |au|^2|bu|^2 - c^2 (Lagrange) is bracketed by 0.99999 - c^2 <= |n|^2 <= 1.00001 - c^2
// (unit vectors to ~1e-7, c to ~5e-7).  The computed t.n is within 1e-5 (bmax + omax) + 1e-6 of
// the exact one (~2e-6 (bmax + omax) by the float error of the cross and dot products), and the
// coordinate bound mag of far_from_lines uses tl <= |b0|_1 + |o|_1, so its margins split into a
// beam part (staged: Ab, Eb) and a lane part (Al, El):
//   reject  <=>  tn > (Eb + El) + (Ab + Al) * (sqrt(nn_hi) * 1.000001 + 1e-6)
// which implies the line-line distance exceeds maxd * 1.0001 + 2 eps with eps >= far_from_lines'
// eps: the same proof that every reference-computed distance of the pair is >= maxd.  Near-parallel
// pairs (|n|^2 possibly < 1e-2) and zero-length segments (El = FLT_MAX) are never rejected.
struct ScanLane {
    f3 q;       // o x au
    float al;   // 2e-5 (omax + 10 |o|_1)
    float el;   // 1e-5 omax, FLT_MAX for a zero-length segment
};

__device__ __forceinline__ ScanLane make_scan_lane(const Lane &L) {
    ScanLane S;
    S.q = mk(L.o.y * L.au.z - L.o.z * L.au.y, L.o.z * L.au.x - L.o.x * L.au.z, L.o.x * L.au.y - L.o.y * L.au.x);
    const float o1 = fabsf(L.o.x) + fabsf(L.o.y) + fabsf(L.o.z);
    S.al = 2e-5f * (L.omax + 10.0f * o1);
    S.el = L.mag_a == 0.0f ? FLT_MAX : 1e-5f * L.omax;
    return S;
}

__device__ __forceinline__ bool scan_far(const ScanLane &S, f3 au, f3 bu, f3 m0, float ab, float eb) {
    const float c = __builtin_fmaf(au.x, bu.x, __builtin_fmaf(au.y, bu.y, au.z * bu.z));
    const float nn_lo = __builtin_fmaf(-c, c, 0.99999f);
    if (!(nn_lo >= 1e-2f)) return false;
    const float x = __builtin_fmaf(au.x, m0.x, __builtin_fmaf(au.y, m0.y, au.z * m0.z));
    const float tn = fabsf(__builtin_fmaf(-bu.x, S.q.x, __builtin_fmaf(-bu.y, S.q.y, __builtin_fmaf(-bu.z, S.q.z, x))));
    const float nl = __builtin_amdgcn_sqrtf(__builtin_fmaf(-c, c, 1.00001f)) * 1.000001f + 1e-6f;
    return tn > __builtin_fmaf(ab + S.al, nl, eb + S.el);
}

constexpr int kTileBlock = 256;  // 4 waves
constexpr int kQueueCap = 128;   // >= 63 left over + 64 appended by one beam / one flush
constexpr int kTileMax = 32;     // beams staged in LDS at a time (longer leaves go in chunks; 64 costs occupancy)

struct TileShared {
    float4 tile[kTileMax][4];  // staged BeamRec lines of the current leaf chunk
    float acc[3][64];          // per-segment RGB accumulators
    int32_t cnt[64];           // per-segment contribution counts (counters only)
    uint16_t q0[kQueueCap];    // box-hit queue: tile slot | segment lane << 8
    int32_t qb1[kQueueCap];    // prefilter-survivor queue: beam index
    uint8_t ql1[kQueueCap];    //                           segment lane
    int32_t stk[kStackDepth];
};

__device__ __forceinline__ float lane_f(float v, int src) { return __shfl(v, src); }

// Stage 3: exact closest points + kernel for n queued pairs (one per lane; all lanes call).
template <bool COUNT>
__device__ __forceinline__ void tile_exact(TileShared &sh, const Lane &M, int first, int n,
                                           const BeamRec *__restrict__ recs, const float4 *__restrict__ pw, float R,
                                           Prof &pf) {
    const int lane = threadIdx.x & 63;
    const bool on = lane < n;
    const int e = (first + (on ? lane : 0)) & (kQueueCap - 1);  // FIFO ring
    const int32_t b = sh.qb1[e];
    const int sl = sh.ql1[e];
    // the pair's segment, from its owner lane's registers
    const f3 o = mk(lane_f(M.o.x, sl), lane_f(M.o.y, sl), lane_f(M.o.z, sl));
    const f3 p = mk(lane_f(M.p.x, sl), lane_f(M.p.y, sl), lane_f(M.p.z, sl));
    const f3 au = mk(lane_f(M.au.x, sl), lane_f(M.au.y, sl), lane_f(M.au.z, sl));
    const float mag_a = lane_f(M.mag_a, sl);
    const BeamV r = load_beam(recs, b);
    if (COUNT && lane == 0) ++pf.ccp_waves;
    if (on) {
        const float maxd = R + r.radius;  // MaxDistance = currentBeamRadius + beam->radius
        float dist;
        const bool ok = closest_distance(o, p, au, mag_a, r.b0, r.bu, r.mag_b, dist);
        if (ok & (dist < maxd)) {
            const float rr = dist / maxd;
            const float w = sqrtf(1.0f - rr * rr);
            const float4 pv = pw[b];
            atomicAdd(&sh.acc[0][sl], pv.x * w);
            atomicAdd(&sh.acc[1][sl], pv.y * w);
            atomicAdd(&sh.acc[2][sl], pv.z * w);
            if (COUNT) atomicAdd(&sh.cnt[sl], 1);
        }
    }
}

// Prefilter-first stage 2: the reference's box test on the beam's (group) box, then exact closest
// points + kernel, for n queued prefilter survivors (one per lane; all lanes call).  The pair's
// beam line comes from L2 (the staged tile may already be replaced).
template <bool COUNT>
__device__ __forceinline__ void tile_box_exact(TileShared &sh, const Lane &M, int first, int n,
                                               const BeamRec *__restrict__ recs, const float4 *__restrict__ pw,
                                               float R, const float *__restrict__ sd, int64_t seg0, Prof &pf,
                                               int dbg = 0) {
    const int lane = threadIdx.x & 63;
    const bool on = lane < n;
    const int e = (first + (on ? lane : 0)) & (kQueueCap - 1);  // FIFO ring
    const int32_t b = sh.qb1[e];
    const int sl = sh.ql1[e];
    const f3 o = mk(lane_f(M.o.x, sl), lane_f(M.o.y, sl), lane_f(M.o.z, sl));
    const f3 invs = mk(lane_f(M.invs.x, sl), lane_f(M.invs.y, sl), lane_f(M.invs.z, sl));
    const float tmax = lane_f(M.tmax, sl);
    const BeamV r = load_beam(recs, b);
    if (COUNT && lane == 0) ++pf.ccp_waves;
    float te;
    bool hit = on & node_test(r.box, o, invs, tmax, te);
    const bool inf = __shfl((int)M.has_inf, sl) != 0;
    if (__ballot(on & inf) != 0ull) {
        if (on & inf) {
            // the rare axis-parallel ray: its direction is re-read (keeps Lane::d out of registers)
            const int64_t so = seg0 + sl;
            const f3 d = mk(sd[3 * so], sd[3 * so + 1], sd[3 * so + 2]);
            const f3 inv = mk(1 / d.x, 1 / d.y, 1 / d.z);
            hit = slab_test(r.box, o, inv, inv.x < 0, inv.y < 0, inv.z < 0, tmax, nullptr);
        }
    }
    if (__ballot(hit) == 0ull) return;
    if (dbg == 3) {  // timing-only: queue, shuffles, beam load and box test, no closest points
        if (hit) atomicAdd(&sh.acc[0][sl], r.radius);
        return;
    }
    // the power load is issued ahead of the closest-point arithmetic (most box hits contribute)
    const float4 pv = hit ? pw[b] : make_float4(0.f, 0.f, 0.f, 0.f);
    const f3 p = mk(lane_f(M.p.x, sl), lane_f(M.p.y, sl), lane_f(M.p.z, sl));
    const f3 au = mk(lane_f(M.au.x, sl), lane_f(M.au.y, sl), lane_f(M.au.z, sl));
    const float mag_a = lane_f(M.mag_a, sl);
    if (hit) {
        const float maxd = R + r.radius;  // MaxDistance = currentBeamRadius + beam->radius
        float dist;
        const bool ok = closest_distance(o, p, au, mag_a, r.b0, r.bu, r.mag_b, dist);
        if (ok & (dist < maxd)) {
            const float rr = dist / maxd;
            const float w = sqrtf(1.0f - rr * rr);
            atomicAdd(&sh.acc[0][sl], pv.x * w);
            atomicAdd(&sh.acc[1][sl], pv.y * w);
            atomicAdd(&sh.acc[2][sl], pv.z * w);
            if (COUNT) atomicAdd(&sh.cnt[sl], 1);
        }
    }
}

// Stage 2: prefilter n box-hit pairs of the staged tile (one per lane; all lanes call); the
// survivors are appended to queue 1, which is drained in batches of 64.  Without the prefilter,
// every pair is forwarded.
template <bool COUNT, bool PREF>
__device__ __forceinline__ void tile_filter(TileShared &sh, const Lane &M, int first, int n, int64_t tile0, int &h1, int &t1,
                                            const BeamRec *__restrict__ recs, const float4 *__restrict__ pw, float R,
                                            Prof &pf) {
    const int lane = threadIdx.x & 63;
    const bool on = lane < n;
    const int e = (first + (on ? lane : 0)) & (kQueueCap - 1);  // FIFO ring
    const unsigned qv = sh.q0[e];
    const int j = (int)(qv & 0xffu), sl = (int)(qv >> 8);
    bool need = on;
    if (PREF) {
        const f3 o = mk(lane_f(M.o.x, sl), lane_f(M.o.y, sl), lane_f(M.o.z, sl));
        const f3 au = mk(lane_f(M.au.x, sl), lane_f(M.au.y, sl), lane_f(M.au.z, sl));
        const float mag_a = lane_f(M.mag_a, sl);
        const float omax = lane_f(M.omax, sl);
        const float4 y = sh.tile[j][1], z = sh.tile[j][2], wv = sh.tile[j][3];
        need = on && !far_from_lines_fast(o, au, mag_a, omax, mk(y.z, y.w, z.x), mk(z.y, z.z, z.w), R + wv.y);
        if (COUNT) pf.rejects += on & !need;
    }
    const unsigned long long m = __ballot(need);
    if (m == 0ull) return;
    if (need) {
        const int pos = (t1 + lanes_below(m)) & (kQueueCap - 1);
        sh.qb1[pos] = (int32_t)(tile0 + j);
        sh.ql1[pos] = (uint8_t)sl;
    }
    t1 += __popcll(m);
    __builtin_amdgcn_wave_barrier();
    if (t1 - h1 >= 64) {
        // FIFO: survivors are evaluated in queue order, so a segment's contributions are summed
        // in the same order with or without the prefilter (bit-identical results)
        tile_exact<COUNT>(sh, M, h1, 64, recs, pw, R, pf);
        h1 += 64;
        if (h1 >= 1024) {
            h1 -= 1024;
            t1 -= 1024;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

template <bool COUNT, bool PREF, int MINW, bool PFIRST>
__global__ __launch_bounds__(kTileBlock, MINW) void k_gather_tile(
    int64_t nseg, const float *__restrict__ so, const float *__restrict__ sp_, const float *__restrict__ sd,
    const float *__restrict__ stmax, float R, float *__restrict__ partial, int32_t *__restrict__ pcnt,
    const BeamRec *__restrict__ recs, const float4 *__restrict__ pw, const Node *__restrict__ nodes, int64_t nvalid,
    int leaf_size, const int32_t *__restrict__ roots, int S, DevCounters *ctr, int dbg,
    const uint8_t *__restrict__ redo) {
    __shared__ TileShared shm[kTileBlock / 64];
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
    if (sub >= roots[S]) return;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    TileShared &sh = shm[w];
    const int64_t s = grp * kTileBlock + threadIdx.x;
    const int64_t seg0 = grp * kTileBlock + (int64_t)__builtin_amdgcn_readfirstlane(w) * 64;  // lane 0 of this wave
    // behind kernel 3 (auto), only the packets it handed over run here; the test is per wave (one
    // packet), so a ragged last packet keeps all 64 lanes (tile staging and shuffles need them)
    if (redo) {
        const int64_t pk = (grp * kTileBlock + (int64_t)w * 64) >> 6;
        if (pk * 64 >= nseg || !redo[pk]) return;
    }
    Lane L;
    const bool valid = load_lane(s, nseg, so, sp_, sd, stmax, L);
    Bundle K;
    K.delta = FLT_MAX;
    if (PFIRST && PREF && __ballot(valid) != 0ull) K = make_bundle(L, valid);
    const ScanLane SL = PFIRST ? make_scan_lane(L) : ScanLane{};
    sh.acc[0][lane] = 0.f;
    sh.acc[1][lane] = 0.f;
    sh.acc[2][lane] = 0.f;
    sh.cnt[lane] = 0;
    __builtin_amdgcn_wave_barrier();
    const bool any_inf = __ballot(L.has_inf) != 0ull;  // some lane has an axis-parallel direction
    int cand = 0;
    unsigned long long visits = 0;
    Prof pf;
    int h0 = 0, t0 = 0, h1 = 0, t1 = 0;  // wave-uniform FIFO ring heads / tails

    // scan one leaf: its beam lines are staged in LDS kTileMax at a time; per lane the reference
    // box test, hits queued; full batches, and each chunk's remainder, go through the filter
    const auto leaf = [&](int32_t c, bool lane_on) {
        const int64_t first = (int64_t)(~c) * leaf_size;
        const int cnt = (int)min((int64_t)leaf_size, nvalid - first);
        if (COUNT) {
            ++pf.leaves;
            pf.beams += cnt;
        }
        if (dbg == 1) return;  // timing-only: traversal without leaf work
        for (int base = 0; base < cnt; base += kTileMax) {
            const int nb = min(kTileMax, cnt - base);
            const int64_t tile0 = first + base;
            __builtin_amdgcn_wave_barrier();
            if (PFIRST) {
                // lane j stages beam j in the scan layout (see ScanLane): (b0, maxd), (bu, Ab),
                // (m0 = bu x b0, Eb); the exact stage reads the beam record itself from L2
                if (lane < nb) {
                    const BeamV r = load_beam(recs, tile0 + lane);
                    const float maxd = R + r.radius;
                    const f3 m0 = mk(r.bu.y * r.b0.z - r.bu.z * r.b0.y, r.bu.z * r.b0.x - r.bu.x * r.b0.z,
                                     r.bu.x * r.b0.y - r.bu.y * r.b0.x);
                    const float bmax = fmaxf(fmaxf(fabsf(r.b0.x), fabsf(r.b0.y)), fabsf(r.b0.z));
                    const float b1 = fabsf(r.b0.x) + fabsf(r.b0.y) + fabsf(r.b0.z);
                    const float ab = maxd * 1.0001f + 2e-5f * (bmax + 10.0f * b1) + 2e-6f;
                    const float eb = 1e-5f * bmax + 1e-6f;
                    sh.tile[lane][0] = make_float4(r.b0.x, r.b0.y, r.b0.z, maxd);
                    sh.tile[lane][1] = make_float4(r.bu.x, r.bu.y, r.bu.z, ab);
                    sh.tile[lane][2] = make_float4(m0.x, m0.y, m0.z, eb);
                }
            } else {
                // 64 lanes copy nb lines of 4 x 16 B: item r -> (beam r >> 1, half r & 1)
                for (int r = lane; r < 2 * nb; r += 64) {
                    const int bj = r >> 1, h = (r & 1) * 2;
                    const float4 *q = reinterpret_cast<const float4 *>(recs + tile0 + bj);
                    const float4 u = q[h], v = q[h + 1];
                    sh.tile[bj][h] = u;
                    sh.tile[bj][h + 1] = v;
                }
            }
            __builtin_amdgcn_wave_barrier();
            if (PFIRST) {
                // prefilter first: per lane and beam only the conservative line-distance bound
                // (lanes that miss the tile's node box miss every beam box in it); survivors go
                // to queue 1 with their global beam index and run box test + exact 64 at a time.
                // Queue order is (leaf, beam, lane) as in the box-first order, so each segment
                // sums the same pairs in the same order (bit-identical to tile_mode 0).
                // packet-level bundle reject, one beam per lane (see make_bundle): beams far from
                // every segment of the packet are skipped by all lanes
                unsigned long long km = ~0ull;
                if (PREF) {
                    bool keep = false;
                    if (lane < nb) {
                        const float4 x = sh.tile[lane][0], y = sh.tile[lane][1];
                        keep = !bundle_far(K, mk(x.x, x.y, x.z), mk(y.x, y.y, y.z), x.w);
                    }
                    km = __ballot(keep);
                }
                unsigned long long todo = COUNT ? (nb >= 64 ? ~0ull : ((1ull << nb) - 1ull))
                                                : (km & (nb >= 64 ? ~0ull : ((1ull << nb) - 1ull)));
                if (COUNT) pf.useful += __popcll(km & (nb >= 64 ? ~0ull : ((1ull << nb) - 1ull)));
                // queue the (beam, lane) survivors of beam j; drain 64 at a time (ring < 128)
                const auto push = [&](int j, bool need) {
                    const unsigned long long m = __ballot(need);
                    if (m == 0ull) return;
                    if (need) {
                        const int pos = (t1 + lanes_below(m)) & (kQueueCap - 1);
                        sh.qb1[pos] = (int32_t)(tile0 + j);
                        sh.ql1[pos] = (uint8_t)lane;
                    }
                    t1 += __popcll(m);
                    __builtin_amdgcn_wave_barrier();
                    if (t1 - h1 >= 64) {
                        if (dbg != 2) tile_box_exact<COUNT>(sh, L, h1, 64, recs, pw, R, sd, seg0, pf, dbg);
                        h1 += 64;
                        if (h1 >= 1024) {
                            h1 -= 1024;
                            t1 -= 1024;
                        }
                        __builtin_amdgcn_wave_barrier();
                    }
                };
                if (!COUNT && PREF) {
                    // two kept beams per step: independent LDS reads and prefilters (ILP), then the
                    // survivors are queued beam by beam in order
                    while (todo != 0ull) {
                        const int j1 = __ffsll((long long)todo) - 1;
                        todo &= todo - 1ull;
                        const bool two = todo != 0ull;
                        const int j2 = two ? __ffsll((long long)todo) - 1 : j1;
                        if (two) todo &= todo - 1ull;
                        const float4 y1 = sh.tile[j1][1], z1 = sh.tile[j1][2];
                        const float4 y2 = sh.tile[j2][1], z2 = sh.tile[j2][2];
                        const bool n1 = lane_on && !scan_far(SL, L.au, mk(y1.x, y1.y, y1.z), mk(z1.x, z1.y, z1.z), y1.w, z1.w);
                        const bool n2 = two && lane_on &&
                                        !scan_far(SL, L.au, mk(y2.x, y2.y, y2.z), mk(z2.x, z2.y, z2.z), y2.w, z2.w);
                        push(j1, n1);
                        if (two) push(j2, n2);
                    }
                    continue;
                }
                while (todo != 0ull) {
                    const int j = __ffsll((long long)todo) - 1;
                    todo &= todo - 1ull;
                    bool need = lane_on && ((km >> j) & 1ull);
                    if (PREF) {
                        const float4 y = sh.tile[j][1], z = sh.tile[j][2];
                        need = need && !scan_far(SL, L.au, mk(y.x, y.y, y.z), mk(z.x, z.y, z.z), y.w, z.w);
                    }
                    if (COUNT) {
                        const Box6 box = load_beam(recs, tile0 + j).box;
                        float te;
                        bool hit = lane_on & node_test(box, L.o, L.invs, L.tmax, te);
                        if (L.has_inf) hit = lane_on & slab_test(box, L.o, L.inv, L.n0, L.n1, L.n2, L.tmax, nullptr);
                        cand += hit;
                        pf.rejects += hit & !need;
                    }
                    push(j, need);
                }
                continue;
            }
            for (int j = 0; j < nb; ++j) {
                const float4 x = sh.tile[j][0], y = sh.tile[j][1];
                const Box6 box{x.x, x.y, x.z, x.w, y.x, y.y};
                float te;
                bool hit = lane_on & node_test(box, L.o, L.invs, L.tmax, te);
                if (any_inf) {
                    if (L.has_inf) hit = lane_on & slab_test(box, L.o, L.inv, L.n0, L.n1, L.n2, L.tmax, nullptr);
                }
                if (COUNT) cand += hit;
                const unsigned long long m = __ballot(hit);
                if (m == 0ull) continue;
                if (COUNT) ++pf.useful;
                if (hit) sh.q0[(t0 + lanes_below(m)) & (kQueueCap - 1)] = (uint16_t)(j | (lane << 8));
                t0 += __popcll(m);
                if (t0 - h0 >= 64) {
                    __builtin_amdgcn_wave_barrier();
                    if (dbg != 2) tile_filter<COUNT, PREF>(sh, L, h0, 64, tile0, h1, t1, recs, pw, R, pf);
                    h0 += 64;
                    __builtin_amdgcn_wave_barrier();
                }
            }
            if (t0 > h0) {
                __builtin_amdgcn_wave_barrier();
                if (dbg != 2) tile_filter<COUNT, PREF>(sh, L, h0, t0 - h0, tile0, h1, t1, recs, pw, R, pf);
            }
            h0 = t0 = 0;  // the chunk's queue is drained (its entries index this chunk's tile)
        }
    };

    if (__ballot(valid) != 0ull) {
        const int32_t root = roots[sub];
        if (root < 0) {
            leaf(root, valid);
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
                bool go0 = m0 != 0ull, go1 = m1 != 0ull;
                if (go0 && c0 < 0) {
                    leaf(c0, h0);
                    go0 = false;
                }
                if (go1 && c1 < 0) {
                    leaf(c1, h1);
                    go1 = false;
                }
                if (go0 && go1) {
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
                        if (lane == 0) atomicOr(&ctr->flags, 1u);
                        break;
                    }
                    sh.stk[sp] = far;
                    ++sp;
                    node = near;
                } else if (go0) {
                    node = c0;
                } else if (go1) {
                    node = c1;
                } else {
                    if (sp == 0) break;
                    --sp;
                    node = sh.stk[sp];
                }
            }
        }
        // drain the prefilter survivors
        __builtin_amdgcn_wave_barrier();
        if (dbg != 2 && t1 > h1) {
            if (PFIRST) tile_box_exact<COUNT>(sh, L, h1, t1 - h1, recs, pw, R, sd, seg0, pf, dbg);
            else tile_exact<COUNT>(sh, L, h1, t1 - h1, recs, pw, R, pf);
        }
        h1 = t1 = 0;
    }
    __builtin_amdgcn_wave_barrier();
    if (valid) {
        float *dst = partial + 3 * ((int64_t)sub * nseg + s);
        dst[0] = sh.acc[0][lane];
        dst[1] = sh.acc[1][lane];
        dst[2] = sh.acc[2][lane];
        if (COUNT) {
            pcnt[2 * ((int64_t)sub * nseg + s)] = cand;
            pcnt[2 * ((int64_t)sub * nseg + s) + 1] = sh.cnt[lane];
        }
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
        }
    }
}

// Sum the per-subtree partials of each segment in subtree order; write seg_rgb and add the
// segment's sum to its pixel (one float atomic per channel, PhotonBeamPixel::Ld +=).  With
// counters, also sum the per-subtree candidate / contribution counts.
__global__ __launch_bounds__(256) void k_reduce(int64_t nseg, const float *__restrict__ partial,
                                                const int32_t *__restrict__ pcnt, const int32_t *__restrict__ roots,
                                                int S, const int32_t *__restrict__ pixel, int64_t npix,
                                                float *__restrict__ accum, float *__restrict__ seg_rgb,
                                                int32_t *__restrict__ seg_counts, DevCounters *ctr,
                                                const uint8_t *__restrict__ redo, const int32_t *__restrict__ roots2) {
    const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const bool in = s < nseg;
    // packets handed over to the second tree (auto mode) hold that tree's subtree partials
    const int nr = (redo && in && redo[s >> 6]) ? roots2[S] : roots[S];
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
        if (seg_rgb) {
            seg_rgb[3 * s] = cr;
            seg_rgb[3 * s + 1] = cg;
            seg_rgb[3 * s + 2] = cb;
        }
        if (seg_counts) {
            seg_counts[2 * s] = (int32_t)c;
            seg_counts[2 * s + 1] = (int32_t)k;
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
    if (pcnt) {
        unsigned long long uc = (unsigned long long)c, uk = (unsigned long long)k;
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
    if (kernel == 3 || kernel == 0) {
        const int64_t packets = (a.nseg + 63) / 64;
        hipError_t em = hipMemsetAsync(a.redo, 0, (size_t)packets, s);
        if (em != hipSuccess) return em;
        const dim3 grid3((unsigned int)(packets * a.split));
#define BRE_LAUNCH_PROXY_W(C, P, W)                                                                              \
    hipLaunchKernelGGL((k_gather_proxy<C, P, W>), grid3, dim3(64), 0, s, a.nseg, a.o, a.p, a.d, a.tmax, a.R,      \
                       a.partial, a.pcnt, a.recs, a.pow, a.nodes, a.nvalid, a.leaf_size, a.roots, a.split,       \
                       a.ctr, a.stack_limit > 0 ? min(a.stack_limit, kProxyStack) : kProxyStack, a.debug_mode,    \
                       a.redo, a.loose_cos > 0.f ? a.loose_cos : kLooseCos)
#define BRE_LAUNCH_PROXY(C, P) BRE_LAUNCH_PROXY_W(C, P, 1)
        if (counters) {
            if (a.prefilter) BRE_LAUNCH_PROXY(true, true);
            else BRE_LAUNCH_PROXY(true, false);
        } else {
            if (a.prefilter) BRE_LAUNCH_PROXY(false, true);
            else BRE_LAUNCH_PROXY(false, false);
        }
#undef BRE_LAUNCH_PROXY
#undef BRE_LAUNCH_PROXY_W
        hipError_t e3 = hipGetLastError();
        if (e3 != hipSuccess) return e3;
    }
    if (kernel == 4 || kernel == 0) {
        // kernel 0 (auto): kernel 3 above on the small-leaf tree, then kernel 4 on the tile tree
        // for the packets kernel 3 handed over (incoherent, or out of LDS stack)
        const bool ho = kernel == 0;
        const Node *nodes4 = ho ? a.nodes2 : a.nodes;
        const int32_t *roots4 = ho ? a.roots2 : a.roots;
        const int leaf4 = ho ? a.leaf2 : a.leaf_size;
        const uint8_t *redo4 = ho ? a.redo : nullptr;
        const dim3 grid4((unsigned int)(((a.nseg + kTileBlock - 1) / kTileBlock) * a.split));
#define BRE_LAUNCH_TILE_W(C, P, W, F)                                                                             \
    hipLaunchKernelGGL((k_gather_tile<C, P, W, F>), grid4, dim3(kTileBlock), 0, s, a.nseg, a.o, a.p, a.d, a.tmax, a.R, \
                       a.partial, a.pcnt, a.recs, a.pow, nodes4, a.nvalid, leaf4, roots4, a.split,                   \
                       a.ctr, a.debug_mode, redo4)
#define BRE_LAUNCH_TILE(C, P)                      \
    do {                                           \
        if (a.tile_mode == 1 && a.occupancy >= 8)  \
            BRE_LAUNCH_TILE_W(C, P, 8, true);      \
        else if (a.tile_mode == 1 && a.occupancy == 7) \
            BRE_LAUNCH_TILE_W(C, P, 7, true);      \
        else if (a.tile_mode == 1)                 \
            BRE_LAUNCH_TILE_W(C, P, 1, true);      \
        else if (a.occupancy >= 8)                 \
            BRE_LAUNCH_TILE_W(C, P, 8, false);     \
        else                                       \
            BRE_LAUNCH_TILE_W(C, P, 1, false);     \
    } while (0)
        if (counters) {
            if (a.prefilter) BRE_LAUNCH_TILE(true, true);
            else BRE_LAUNCH_TILE(true, false);
        } else {
            if (a.prefilter) BRE_LAUNCH_TILE(false, true);
            else BRE_LAUNCH_TILE(false, false);
        }
#undef BRE_LAUNCH_TILE
#undef BRE_LAUNCH_TILE_W
        hipError_t e4 = hipGetLastError();
        if (e4 != hipSuccess) return e4;
        hipLaunchKernelGGL(k_reduce, dim3((unsigned int)((a.nseg + 255) / 256)), dim3(256), 0, s, a.nseg, a.partial,
                           counters ? a.pcnt : nullptr, a.roots, a.split, a.pixel, a.npix, a.accum, a.seg_rgb,
                           counters ? a.seg_counts : nullptr, a.ctr, redo4, a.roots2);
        return hipGetLastError();
    }
    const int64_t groups = (a.nseg + kWaveBlock - 1) / kWaveBlock;
    const dim3 grid((unsigned int)(groups * a.split));
    const uint8_t *redo = kernel == 3 ? a.redo : nullptr;  // kernel 1 as kernel 3's device-side fallback
#define BRE_LAUNCH_WAVE(C, P)                                                                                   \
    hipLaunchKernelGGL((k_gather_wave<C, P>), grid, dim3(kWaveBlock), 0, s, a.nseg, a.o, a.p, a.d, a.tmax, a.R, \
                       a.partial, a.pcnt, a.recs, a.pow, a.nodes, a.nvalid, a.leaf_size, a.roots, a.split,        \
                       a.ctr, a.debug_mode, redo)
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
                       counters ? a.pcnt : nullptr, a.roots, a.split, a.pixel, a.npix, a.accum, a.seg_rgb,
                       counters ? a.seg_counts : nullptr, a.ctr, nullptr, nullptr);
    return hipGetLastError();
}

hipError_t launch_zero_outputs(const GatherArgs &a, hipStream_t s) {
    if (a.nseg == 0 || (!a.seg_rgb && !a.seg_counts)) return hipSuccess;
    hipLaunchKernelGGL(k_zero_seg, dim3((unsigned int)((a.nseg + 255) / 256)), dim3(256), 0, s, a.nseg, a.seg_rgb,
                       a.seg_counts);
    return hipGetLastError();
}

}  // namespace bre
