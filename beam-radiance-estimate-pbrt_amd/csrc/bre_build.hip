// bre_build.hip — GPU build of the beam BVH for gfx950.
//
// Replaces the reference's single-threaded SAH build (PhotonBeamBVH ctor + recursiveBuild +
// flattenBVH2Tree, src/core/photonbeambvh.cpp:204-248, 259-425, 663-681) with a Karras-style
// linear BVH over 63-bit Morton codes of the beam-box centroids — the GPU form of the
// reference's own (unused) HLBVH path (EncodeMorton3 / RadixSort / emitLBVH2, :109-182, 427-559).
//
// The tree shape does not have to match the reference: the set of beams gathered for a
// segment is the set whose *own test box* passes Bounds3::IntersectP (see DESIGN.md "key
// enabler").  The one place where the reference's tree leaks into that set is a leaf holding
// several beams, which recursiveBuild creates exactly for beams with bit-identical centroids
// (:289-297); their leaf box (the union) is what the reference tests.  k_pack reproduces that by
// giving every beam the union box of its equal-centroid group.
//
// Passes (all on the context stream):
//   k_prep      per beam: WorldBound box (reference arithmetic), centroid, validity, centroid and
//               end-point bounds
//   k_morton    per beam: 63-bit Morton key of the centroid (invalid beams sort last)
//   radix sort  rocPRIM radix_sort_pairs (key, beam index)
//   k_group     (tree key 1) per beam: its equal-centroid group box, found in centroid order
//   k_morton_se (tree key 1) per beam: 60-bit Morton key of (start, end), sorted again: the tree order
//   k_pack      per sorted beam: (group) box, 64-B BeamRec, scaled power
//   k_karras    per interior node: Karras 2012 split over leaf clusters of `leaf_size` beams
//   k_refit     per leaf cluster: bottom-up union of child boxes (agent-scope release/acquire
//               hand-off through one counter per node, cdna_hip_programming.md Guideline 16)
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <float.h>

#include <algorithm>

#include "bre_device.h"
#include "bre_math.h"

namespace bre {

namespace {

__device__ __forceinline__ unsigned int f2ord(float f) {
    unsigned int u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(unsigned int u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

__device__ __forceinline__ bool finite6(const float *b) {
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 6; ++k) ok = ok && isfinite(b[k]);
    return ok;
}

#ifndef BRE_PASS_BLOCK
#define BRE_PASS_BLOCK 64  // one wave (bre_slot.hip; 256 until round 5)
#endif
constexpr int kBlock = BRE_PASS_BLOCK;  // threads per block of the pass kernels

__global__ void k_prep_init(unsigned int *__restrict__ cbounds, unsigned int *__restrict__ nvalid) {
    const int t = threadIdx.x;
    if (t < 12) cbounds[t] = ((t / 3) & 1) ? 0u : 0xffffffffu;  // min, max, min, max
    if (t < 3) nvalid[t] = t == 1 ? 0xffffffffu : 0u;
}

// Grid-stride: each thread prepares several beams and keeps running centroid bounds; the block
// reduces them (wave shuffles, then LDS across its 4 waves) and issues one set of atomics, so the
// 7 contended global atomics are paid per block, not per wave (~3 ms -> ~0.2 ms at 2.7M beams).
__global__ __launch_bounds__(kBlock) void k_prep(const float *__restrict__ start, const float *__restrict__ end,
                                                 const float *__restrict__ radius, int64_t n, int sqrt_mode,
                                                 float *__restrict__ box, float *__restrict__ cent,
                                                 unsigned int *__restrict__ cbounds, unsigned int *__restrict__ nvalid) {
    __shared__ unsigned int red[kBlock / 64][15];
    // ordered-uint min (lo) / max (hi) of valid centroids and of valid beams' end points; identity values
    unsigned int mn[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu};
    unsigned int mx[3] = {0u, 0u, 0u};
    unsigned int emn[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu};
    unsigned int emx[3] = {0u, 0u, 0u};
    unsigned int cnt = 0;
    unsigned int rmn = 0xffffffffu, rmx = 0u;  // min / max of the valid beams' radius bits
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        const f3 s = mk(start[3 * i], start[3 * i + 1], start[3 * i + 2]);
        const f3 e = mk(end[3 * i], end[3 * i + 1], end[3 * i + 2]);
        const float rad = radius[i];
        f3 lo, hi;
        world_bound(s, e, rad, sqrt_mode, lo, hi);
        float b[6] = {lo.x, lo.y, lo.z, hi.x, hi.y, hi.z};
#pragma unroll
        for (int k = 0; k < 6; ++k) box[6 * i + k] = b[k];
        // centroid = .5f * pMin + .5f * pMax  (photonbeambvh.cpp:51-54)
        const f3 c = add3(scale3(lo, .5f), scale3(hi, .5f));
        cent[3 * i] = c.x;
        cent[3 * i + 1] = c.y;
        cent[3 * i + 2] = c.z;
        const bool valid = finite6(b) && isfinite(c.x) && isfinite(c.y) && isfinite(c.z);
        if (valid) {
            const unsigned int u[3] = {f2ord(c.x), f2ord(c.y), f2ord(c.z)};
            const unsigned int us[3] = {f2ord(s.x), f2ord(s.y), f2ord(s.z)};
            const unsigned int ue[3] = {f2ord(e.x), f2ord(e.y), f2ord(e.z)};
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                mn[k] = min(mn[k], u[k]);
                mx[k] = max(mx[k], u[k]);
                emn[k] = min(emn[k], min(us[k], ue[k]));
                emx[k] = max(emx[k], max(us[k], ue[k]));
            }
            rmn = min(rmn, __float_as_uint(rad));
            rmx = max(rmx, __float_as_uint(rad));
            ++cnt;
        }
    }
    // wave reduction (64 lanes), then across the block's waves in LDS, then one set of atomics
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            mn[k] = min(mn[k], (unsigned int)__shfl_xor((int)mn[k], off));
            mx[k] = max(mx[k], (unsigned int)__shfl_xor((int)mx[k], off));
            emn[k] = min(emn[k], (unsigned int)__shfl_xor((int)emn[k], off));
            emx[k] = max(emx[k], (unsigned int)__shfl_xor((int)emx[k], off));
        }
        cnt += (unsigned int)__shfl_xor((int)cnt, off);
        rmn = min(rmn, (unsigned int)__shfl_xor((int)rmn, off));
        rmx = max(rmx, (unsigned int)__shfl_xor((int)rmx, off));
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            red[w][k] = mn[k];
            red[w][3 + k] = mx[k];
            red[w][7 + k] = emn[k];
            red[w][10 + k] = emx[k];
        }
        red[w][6] = cnt;
        red[w][13] = rmn;
        red[w][14] = rmx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int v = 1; v < kBlock / 64; ++v) {
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                mn[k] = min(mn[k], red[v][k]);
                mx[k] = max(mx[k], red[v][3 + k]);
                emn[k] = min(emn[k], red[v][7 + k]);
                emx[k] = max(emx[k], red[v][10 + k]);
            }
            cnt += red[v][6];
            rmn = min(rmn, red[v][13]);
            rmx = max(rmx, red[v][14]);
        }
        if (cnt != 0u) {
            atomicAdd(nvalid, cnt);
            atomicMin(&nvalid[1], rmn);
            atomicMax(&nvalid[2], rmx);
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                atomicMin(&cbounds[k], mn[k]);
                atomicMax(&cbounds[3 + k], mx[k]);
                atomicMin(&cbounds[6 + k], emn[k]);
                atomicMax(&cbounds[9 + k], emx[k]);
            }
        }
    }
}

__device__ __forceinline__ unsigned long long expand21(unsigned int v) {
    unsigned long long x = v & 0x1fffffull;
    x = (x | (x << 32)) & 0x1f00000000ffffull;
    x = (x | (x << 16)) & 0x1f0000ff0000ffull;
    x = (x | (x << 8)) & 0x100f00f00f00f00full;
    x = (x | (x << 4)) & 0x10c30c30c30c30c3ull;
    x = (x | (x << 2)) & 0x1249249249249249ull;
    return x;
}

__global__ __launch_bounds__(kBlock) void k_morton(const float *__restrict__ box, const float *__restrict__ cent,
                                                   const unsigned int *__restrict__ cbounds, int64_t n,
                                                   unsigned long long *__restrict__ keys, int32_t *__restrict__ vals) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    float b[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) b[k] = box[6 * i + k];
    const float c[3] = {cent[3 * i], cent[3 * i + 1], cent[3 * i + 2]};
    unsigned long long key = ~0ull;
    if (finite6(b) && isfinite(c[0]) && isfinite(c[1]) && isfinite(c[2])) {
        unsigned int q[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float lo = ord2f(cbounds[k]), hi = ord2f(cbounds[3 + k]);
            const float ext = hi - lo;
            float u = ext > 0.0f ? (c[k] - lo) / ext : 0.0f;
            u = fminf(fmaxf(u * 2097152.0f, 0.0f), 2097151.0f);
            q[k] = (unsigned int)u;
        }
        key = (expand21(q[2]) << 2) | (expand21(q[1]) << 1) | expand21(q[0]);
    }
    keys[i] = key;
    vals[i] = (int32_t)i;
}

// Tree keys 1 / 2: the centroid sort only has to bring each equal-centroid group together for k_group
// (the tree order comes from the second sort, whose values are the input indices again), so its key is
// a 31-bit hash of the centroid's bits (zeros canonical: -0 == +0 for the group test) and the sort runs
// over 32 bits, four radix passes instead of eight; invalid beams carry 0xffffffff and sort last.  A
// hash collision only lengthens k_group's equal-key run scan, which tests the centroids themselves.
__device__ __forceinline__ unsigned int mix32(unsigned int h) {
    h ^= h >> 16;
    h *= 0x7feb352du;
    h ^= h >> 15;
    h *= 0x846ca68bu;
    h ^= h >> 16;
    return h;
}
__global__ __launch_bounds__(kBlock) void k_cent_hash(const float *__restrict__ box, const float *__restrict__ cent,
                                                      int64_t n, unsigned long long *__restrict__ keys,
                                                      int32_t *__restrict__ vals) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    float b[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) b[k] = box[6 * i + k];
    const float c[3] = {cent[3 * i], cent[3 * i + 1], cent[3 * i + 2]};
    unsigned long long key = 0xffffffffull;
    if (finite6(b) && isfinite(c[0]) && isfinite(c[1]) && isfinite(c[2])) {
        unsigned int u[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) u[k] = c[k] == 0.0f ? 0u : __float_as_uint(c[k]);
        key = mix32(u[0] ^ mix32(u[1] ^ mix32(u[2] + 0x9e3779b9u))) >> 1;
    }
    keys[i] = key;
    vals[i] = (int32_t)i;
}

// Tree order (BuildBuffers::beam_key 1 and 2): a 60-bit key of the beam's start AND
// end point (10 bits each, in the box of all valid beams' end points), so a leaf tile holds beams
// with both ends close -- a coherent bundle of nearly parallel, nearly coincident segments -- instead
// of beams with close centroids and any direction (beam_key 0).  Tiles and the nodes above them are
// then tighter (C2: 4858 -> 3596 beam lines staged per packet wave, 37% -> 45% of them kept by the
// packet rejects, 2.67M -> 3.17M estimates/s, profiles/r3).  Only the tree's shape changes: every
// beam is still tested with its own (group) box.  beam_key 2 (the default) orders the same six
// 10-bit coordinates along a Hilbert curve instead of a Morton curve: consecutive keys never jump
// across the box, so fewer tiles straddle two distant bundles (C2 +2.2%, and +6.4% together with the
// Hilbert segment order, profiles/r3/sweep2).
__device__ __forceinline__ unsigned int q10(float x, float lo, float ext) {
    float u = ext > 0.0f ? (x - lo) / ext : 0.0f;
    u = fminf(fmaxf(u * 1024.0f, 0.0f), 1023.0f);
    return (unsigned int)u;
}
__global__ __launch_bounds__(kBlock) void k_morton_se(const float *__restrict__ box, const float *__restrict__ cent,
                                                      const float *__restrict__ start, const float *__restrict__ end,
                                                      const unsigned int *__restrict__ ebounds, int64_t n,
                                                      int hilbert, unsigned long long *__restrict__ keys,
                                                      int32_t *__restrict__ vals) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    float b[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) b[k] = box[6 * i + k];
    const float c[3] = {cent[3 * i], cent[3 * i + 1], cent[3 * i + 2]};
    unsigned long long key = ~0ull;
    if (finite6(b) && isfinite(c[0]) && isfinite(c[1]) && isfinite(c[2])) {
        unsigned int q[6];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float lo = ord2f(ebounds[k]), hi = ord2f(ebounds[3 + k]);
            q[k] = q10(start[3 * i + k], lo, hi - lo);
            q[3 + k] = q10(end[3 * i + k], lo, hi - lo);
        }
        if (hilbert) {
            key = hilbert_key<6, 10>(q);
        } else {
            key = 0ull;
#pragma unroll
            for (int bit = 9; bit >= 0; --bit)
#pragma unroll
                for (int k = 0; k < 6; ++k) key = (key << 1) | ((q[k] >> bit) & 1u);
        }
    }
    keys[i] = key;
    vals[i] = (int32_t)i;
}

// Equal-centroid groups in centroid-Morton order (the reference's multi-beam SAH leaves,
// photonbeambvh.cpp:289-297): every valid beam's group box (the union of the boxes of the beams with
// a bit-identical centroid; members share the centroid key, so they lie in one equal-key run),
// written in input order for k_pack.
__global__ __launch_bounds__(kBlock) void k_group(const float *__restrict__ box, const float *__restrict__ cent,
                                                  const unsigned long long *__restrict__ keys,
                                                  const int32_t *__restrict__ vals, int64_t nvalid,
                                                  float *__restrict__ gbox) {
    const int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (s >= nvalid) return;
    const int32_t i = vals[s];
    const unsigned long long key = keys[s];
    float lo[3] = {box[6 * i], box[6 * i + 1], box[6 * i + 2]};
    float hi[3] = {box[6 * i + 3], box[6 * i + 4], box[6 * i + 5]};
    const float c0 = cent[3 * i], c1 = cent[3 * i + 1], c2 = cent[3 * i + 2];
    for (int dir = -1; dir <= 1; dir += 2) {
        for (int64_t t = s + dir; t >= 0 && t < nvalid && keys[t] == key; t += dir) {
            const int32_t j = vals[t];
            if (cent[3 * j] == c0 && cent[3 * j + 1] == c1 && cent[3 * j + 2] == c2) {
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    lo[k] = smin(lo[k], box[6 * j + k]);
                    hi[k] = smax(hi[k], box[6 * j + 3 + k]);
                }
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        gbox[6 * i + k] = lo[k];
        gbox[6 * i + 3 + k] = hi[k];
    }
}

// GROUP: the group boxes come from k_group (tree keys 1 / 2), so no centroid or key is read here
template <bool GROUP>
__global__ __launch_bounds__(kBlock) void k_pack(const float *__restrict__ start, const float *__restrict__ end,
                                                 const float *__restrict__ radius, const float *__restrict__ power,
                                                 const float *__restrict__ box, const float *__restrict__ cent,
                                                 const unsigned long long *__restrict__ keys,
                                                 const int32_t *__restrict__ vals, int64_t nvalid,
                                                 const float *__restrict__ gbox, BeamRec *__restrict__ recs,
                                                 float4 *__restrict__ pw, int uniform_radius) {
    const int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (s >= nvalid) return;
    const int32_t i = vals[s];
    const float *bx = GROUP ? gbox : box;  // gbox: the group boxes of k_group (tree keys 1 / 2)
    float lo[3] = {bx[6 * i], bx[6 * i + 1], bx[6 * i + 2]};
    float hi[3] = {bx[6 * i + 3], bx[6 * i + 4], bx[6 * i + 5]};
    if (!GROUP) {
        const unsigned long long key = keys[s];
        const float c0 = cent[3 * i], c1 = cent[3 * i + 1], c2 = cent[3 * i + 2];
        // Tree key 0: the equal-centroid group (the reference's multi-beam SAH leaf), the union of the
        // members' boxes; members share the centroid key, so they are within this key run.
        for (int64_t t = s - 1; t >= 0 && keys[t] == key; --t) {
            const int32_t j = vals[t];
            if (cent[3 * j] == c0 && cent[3 * j + 1] == c1 && cent[3 * j + 2] == c2) {
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    lo[k] = smin(lo[k], box[6 * j + k]);
                    hi[k] = smax(hi[k], box[6 * j + 3 + k]);
                }
            }
        }
        for (int64_t t = s + 1; t < nvalid && keys[t] == key; ++t) {
            const int32_t j = vals[t];
            if (cent[3 * j] == c0 && cent[3 * j + 1] == c1 && cent[3 * j + 2] == c2) {
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    lo[k] = smin(lo[k], box[6 * j + k]);
                    hi[k] = smax(hi[k], box[6 * j + 3 + k]);
                }
            }
        }
    }
    const f3 b0 = mk(start[3 * i], start[3 * i + 1], start[3 * i + 2]);
    const f3 b1 = mk(end[3 * i], end[3 * i + 1], end[3 * i + 2]);
    const f3 B = sub3(b1, b0);
    const float magB = len3(B);
    const f3 bu = div3(B, magB);
    BeamRec r;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        r.lo[k] = lo[k];
        r.hi[k] = hi[k];
    }
    r.b0[0] = b0.x; r.b0[1] = b0.y; r.b0[2] = b0.z;
    r.bu[0] = bu.x; r.bu[1] = bu.y; r.bu[2] = bu.z;
    r.mag_b = magB;
    // `1e-5 * beam->powerEnd` = powerEnd.c[k] * (Float)1e-5  (photonbeam.cpp:504, spectrum.h:165-179)
    const float k5 = 1e-5f;
    const float4 p = make_float4(power[3 * i] * k5, power[3 * i + 1] * k5, power[3 * i + 2] * k5, 0.0f);
    // a uniform-radius set carries the power in the record (BeamRec, BeamSet)
    r.radius = uniform_radius ? p.x : radius[i];
    r.pad[0] = uniform_radius ? p.y : 0.0f;
    r.pad[1] = uniform_radius ? p.z : 0.0f;
    recs[s] = r;
    pw[s] = p;
}

// keys are compared from bit key_lo up: the bits the sort ordered (coarse keys, option 121), so the
// leaves' keys are monotone -- unsorted low bits would give the Karras split a non-monotone sequence
// and an invalid hierarchy
__device__ __forceinline__ int ldelta(const unsigned long long *__restrict__ keys, int leaf_size, int nleaf, int i, int j,
                                      int key_lo) {
    if (j < 0 || j >= nleaf) return -1;
    const unsigned long long ki = keys[(int64_t)i * leaf_size] >> key_lo, kj = keys[(int64_t)j * leaf_size] >> key_lo;
    if (ki == kj) return 64 + __clz((unsigned int)(i ^ j));
    return __clzll(ki ^ kj);
}

__global__ __launch_bounds__(kBlock) void k_karras(const unsigned long long *__restrict__ keys, int leaf_size, int nleaf,
                                                   Node *__restrict__ nodes, int32_t *__restrict__ leaf_parent,
                                                   int key_lo) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= nleaf - 1) return;
    const int d = (ldelta(keys, leaf_size, nleaf, i, i + 1, key_lo) - ldelta(keys, leaf_size, nleaf, i, i - 1, key_lo)) >= 0 ? 1 : -1;
    const int dmin = ldelta(keys, leaf_size, nleaf, i, i - d, key_lo);
    int lmax = 2;
    while (ldelta(keys, leaf_size, nleaf, i, i + lmax * d, key_lo) > dmin) lmax <<= 1;
    int l = 0;
    for (int t = lmax >> 1; t >= 1; t >>= 1)
        if (ldelta(keys, leaf_size, nleaf, i, i + (l + t) * d, key_lo) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = ldelta(keys, leaf_size, nleaf, i, j, key_lo);
    int s = 0, t = l;
    do {
        t = (t + 1) >> 1;
        if (ldelta(keys, leaf_size, nleaf, i, i + (s + t) * d, key_lo) > dnode) s += t;
    } while (t > 1);
    const int gamma = i + s * d + min(d, 0);
    const int lo = min(i, j), hi = max(i, j);
    int32_t left, right;
    if (lo == gamma) {
        left = ~gamma;
        leaf_parent[gamma] = i;
    } else {
        left = gamma;
        nodes[gamma].parent = i;
    }
    if (hi == gamma + 1) {
        right = ~(gamma + 1);
        leaf_parent[gamma + 1] = i;
    } else {
        right = gamma + 1;
        nodes[gamma + 1].parent = i;
    }
    nodes[i].child[0] = left;
    nodes[i].child[1] = right;
    nodes[i].nleaf = hi - lo + 1;
    if (i == 0) nodes[0].parent = -1;
}

__device__ __forceinline__ void leaf_box(const BeamRec *__restrict__ recs, int64_t nvalid, int leaf_size, int c,
                                         float lo[3], float hi[3]) {
    const int64_t first = (int64_t)c * leaf_size;
    const int64_t last = min(first + leaf_size, nvalid);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        lo[k] = FLT_MAX;
        hi[k] = -FLT_MAX;
    }
    for (int64_t b = first; b < last; ++b) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            lo[k] = fminf(lo[k], recs[b].lo[k]);
            hi[k] = fmaxf(hi[k], recs[b].hi[k]);
        }
    }
}

__global__ __launch_bounds__(kBlock) void k_refit(const BeamRec *__restrict__ recs, int64_t nvalid, int leaf_size,
                                                  int nleaf, Node *nodes, const int32_t *__restrict__ leaf_parent,
                                                  unsigned int *visit) {
    const int c = blockIdx.x * kBlock + threadIdx.x;
    if (c >= nleaf) return;
    float lo[3], hi[3];
    leaf_box(recs, nvalid, leaf_size, c, lo, hi);
    int32_t me = ~c;
    int32_t p = leaf_parent[c];
    while (p >= 0) {
        const int slot = (nodes[p].child[0] == me) ? 0 : 1;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            nodes[p].lo[slot][k] = lo[k];
            nodes[p].hi[slot][k] = hi[k];
        }
        // release our slot, then count arrivals at p (Guideline 16: release -> vmcnt(0) -> atomic)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned int old = __hip_atomic_fetch_add(&visit[p], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == 0u) return;  // sibling not done yet; it will carry p upward
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float a = __hip_atomic_load(&nodes[p].lo[0][k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const float b = __hip_atomic_load(&nodes[p].lo[1][k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const float e = __hip_atomic_load(&nodes[p].hi[0][k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const float f = __hip_atomic_load(&nodes[p].hi[1][k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            lo[k] = fminf(a, b);
            hi[k] = fmaxf(e, f);
        }
        me = p;
        p = nodes[p].parent;
    }
}

// Single-leaf tree: one root whose second child is empty.
__global__ void k_single(const BeamRec *__restrict__ recs, int64_t nvalid, int leaf_size, Node *nodes) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    float lo[3], hi[3];
    leaf_box(recs, nvalid, leaf_size, 0, lo, hi);
    Node n;
    for (int k = 0; k < 3; ++k) {
        n.lo[0][k] = lo[k];
        n.hi[0][k] = hi[k];
        n.lo[1][k] = FLT_MAX;
        n.hi[1][k] = -FLT_MAX;
    }
    n.child[0] = ~0;
    n.child[1] = kEmptyChild;
    n.parent = -1;
    n.nleaf = 1;
    nodes[0] = n;
}

inline unsigned int grid_for(int64_t n) { return (unsigned int)((n + kBlock - 1) / kBlock); }

}  // namespace

hipError_t launch_prep(const BuildBuffers &b, hipStream_t s) {
    // cbounds: centroid min = 0xffffffff, max = 0, then end-point min / max; nvalid = 0
    // the reduction targets' identities, one launch: centroid min / max, end-point min / max, then the
    // valid count and the radius bits' min / max
    hipLaunchKernelGGL(k_prep_init, dim3(1), dim3(64), 0, s, b.cbounds, b.nvalid);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (b.n == 0) return hipSuccess;
    // grid-stride over 512 blocks: each block's reduction ends in 14 same-address atomics, which the L2
    // serialises (~70 ns each): 2048 blocks cost ~0.2 ms of them at C2
    const unsigned prep_grid = (unsigned)std::min<int64_t>((int64_t)grid_for(b.n), 512);
    hipLaunchKernelGGL(k_prep, dim3(prep_grid), dim3(kBlock), 0, s, b.start, b.end, b.radius, b.n, b.sqrt_mode,
                       b.box, b.cent, b.cbounds, b.nvalid);
    return hipGetLastError();
}

hipError_t launch_morton(const BuildBuffers &b, hipStream_t s) {
    if (b.n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_morton, dim3(grid_for(b.n)), dim3(kBlock), 0, s, b.box, b.cent, b.cbounds, b.n, b.keys,
                       b.vals);
    return hipGetLastError();
}

hipError_t launch_cent_hash(const BuildBuffers &b, hipStream_t s) {
    if (b.n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_cent_hash, dim3(grid_for(b.n)), dim3(kBlock), 0, s, b.box, b.cent, b.n, b.keys, b.vals);
    return hipGetLastError();
}

hipError_t launch_tree_key(const BuildBuffers &b, int64_t nvalid, hipStream_t s) {
    if (b.n == 0) return hipSuccess;
    if (nvalid > 0)
        hipLaunchKernelGGL(k_group, dim3(grid_for(nvalid)), dim3(kBlock), 0, s, b.box, b.cent, b.keys_alt, b.vals_alt,
                           nvalid, b.gbox);
    hipLaunchKernelGGL(k_morton_se, dim3(grid_for(b.n)), dim3(kBlock), 0, s, b.box, b.cent, b.start, b.end,
                       b.cbounds + 6, b.n, b.beam_key == 2 ? 1 : 0, b.keys, b.vals);
    return hipGetLastError();
}

size_t sort_temp_bytes(int64_t n) {
    size_t bytes = 0;
    (void)rocprim::radix_sort_pairs(nullptr, bytes, (unsigned long long *)nullptr, (unsigned long long *)nullptr,
                              (int32_t *)nullptr, (int32_t *)nullptr, (size_t)n, 0, 64);
    return std::max(bytes, slot_sort_temp_bytes(n, 8));
}

hipError_t launch_sort(const BuildBuffers &b, hipStream_t s, int end_bit, int begin_bit) {
    if (b.n == 0) return hipSuccess;
    size_t bytes = b.sort_tmp_bytes;
    // Morton keys use bits [0, 63), the centroid hash bits [0, 32); invalid beams (~0) sort last either
    // way, also from a begin_bit > 0 (bits 60-63 are set only in theirs)
    if (b.slot) return slot_sort_pairs(b.sort_tmp, b.keys, b.keys_alt, b.vals, b.vals_alt, b.n, begin_bit, end_bit, s);
    return rocprim::radix_sort_pairs(b.sort_tmp, bytes, b.keys, b.keys_alt, b.vals, b.vals_alt, (size_t)b.n,
                                     (unsigned int)begin_bit, (unsigned int)end_bit, s);
}

hipError_t launch_pack(const BuildBuffers &b, int64_t nvalid, hipStream_t s) {
    if (nvalid == 0) return hipSuccess;
    if (b.beam_key >= 1)
        hipLaunchKernelGGL(k_pack<true>, dim3(grid_for(nvalid)), dim3(kBlock), 0, s, b.start, b.end, b.radius, b.power,
                           b.box, b.cent, b.keys_alt, b.vals_alt, nvalid, b.gbox, b.recs, b.pow, b.uniform_radius);
    else
        hipLaunchKernelGGL(k_pack<false>, dim3(grid_for(nvalid)), dim3(kBlock), 0, s, b.start, b.end, b.radius, b.power,
                           b.box, b.cent, b.keys_alt, b.vals_alt, nvalid, nullptr, b.recs, b.pow, b.uniform_radius);
    return hipGetLastError();
}

hipError_t launch_hierarchy(const BuildBuffers &b, int64_t nvalid, hipStream_t s) {
    if (nvalid == 0) return hipSuccess;
    const int K = b.leaf_size;
    if (K < 1) return hipErrorInvalidValue;
    const int64_t nleaf64 = (nvalid + K - 1) / K;
    // the hierarchy writes nleaf - 1 nodes (1 for a single leaf), nleaf leaf parents and nleaf - 1
    // refit counters: refuse buffers sized for another leaf size instead of writing past them
    if (nleaf64 > INT32_MAX || (uint64_t)(nleaf64 > 1 ? nleaf64 - 1 : 1) > b.nodes_cap ||
        (nleaf64 > 1 && ((uint64_t)nleaf64 > b.leaf_parent_cap || (uint64_t)(nleaf64 - 1) > b.visit_cap)))
        return hipErrorInvalidValue;
    const int nleaf = (int)nleaf64;
    if (nleaf == 1) {
        hipLaunchKernelGGL(k_single, dim3(1), dim3(64), 0, s, b.recs, nvalid, K, b.nodes);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_karras, dim3(grid_for(nleaf - 1)), dim3(kBlock), 0, s, b.keys_alt, K, nleaf, b.nodes,
                       b.leaf_parent, b.key_lo);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = b.slot ? slot_fill(b.visit, nleaf - 1, 0u, s) : hipMemsetAsync(b.visit, 0, sizeof(unsigned int) * (size_t)(nleaf - 1), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_refit, dim3(grid_for(nleaf)), dim3(kBlock), 0, s, b.recs, nvalid, K, nleaf, b.nodes,
                       b.leaf_parent, b.visit);
    return hipGetLastError();
}

}  // namespace bre
