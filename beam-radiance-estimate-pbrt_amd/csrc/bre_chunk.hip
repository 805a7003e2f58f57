// bre_chunk.hip — capsule-chunk index and gather (kernel 5) for gfx950.
//
// The reference gathers, for each camera segment, every beam whose quirky WorldBound box the
// segment's ray hits (photonbeambvh.h:60-72, photonbeambvh.cpp:685-723) and then keeps the ones
// with ComputeClosestPoints distance d < R + r (photonbeam.cpp:494-508).  In a box full of fog the
// boxes of long diagonal beams are huge: at C2 a camera segment hits ~16% of all beam boxes while
// only ~1.8% of the beams pass within R + r.  The pixel value depends only on the pairs that
// contribute, so this kernel finds them through a tighter index and then applies the reference's
// own tests to each, unchanged:
//
//   * every beam LINE, clipped to the box of this gather's segments (expanded by E), is cut into
//     chunks of length ~len_factor * E, E = (R + r)(1 + 1e-3) + margin;  each chunk's box is its line
//     piece expanded by E, so it contains every point within R + r of the piece;
//   * a pair contributes only if d < R + r, where d = |pA - pB| with pA on the segment and
//     pB = b0 + bu*s on the beam line (ComputeClosestPoints keeps pB on the LINE when t0 is inside
//     A and t1 is not, photonbeam.cpp:178-181, so s may lie outside [0, |B|]: hence the whole line);
//     the segment's ray therefore hits the box of the chunk whose piece holds pB;
//   * the chunks of one line partition the parameter axis into ownership intervals [s_lo, s_hi)
//     (first and last open to -inf / +inf), and a pair is evaluated in full only by the chunk that
//     owns its s, so each pair is counted once — s is computed by the same instruction sequence
//     from the same inputs wherever the pair is met;
//   * the owning chunk then applies, in this order, d < R + r, the reference's exact slab test on
//     the parent's (group) WorldBound box, and adds 1e-5 * powerEnd * sqrt(1 - (d/(R+r))^2).
//
// So the set of contributing pairs and each pair's value are the reference's bit for bit (the
// same closest-point, box-test and kernel arithmetic as kernels 1-4); only the float summation
// order of a segment's contributions differs, as in every kernel.  What is NOT reproduced is the
// reference's candidate count C (box hits that do not contribute are never enumerated), so
// seg_counts[0] here counts the pairs that reached the exact closest-point code.
//
// The index depends on the segments' box and on R, so it is built per gather (LBVH over chunk
// centroids with the same Morton / Karras / refit kernels as the beam BVH, bre_build.hip).
#include <hip/hip_runtime.h>
#include <rocprim/device/device_scan.hpp>

#include <float.h>

#include "bre_device.h"
#include "bre_lane.h"
#include "bre_math.h"

namespace bre {

namespace {

constexpr int kBlock = 256;
constexpr int kChunkBlock = 128;
constexpr int kChunkStack = 64;
constexpr int kMaxChunksPerBeam = 1 << 16;

__device__ __forceinline__ unsigned int f2ord(float f) {
    unsigned int u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(unsigned int u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

__device__ __forceinline__ void wave_minmax_atomic(unsigned int mn[3], unsigned int mx[3], bool any,
                                                   unsigned int *bounds) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            mn[k] = min(mn[k], (unsigned int)__shfl_xor((int)mn[k], off));
            mx[k] = max(mx[k], (unsigned int)__shfl_xor((int)mx[k], off));
        }
    }
    if ((threadIdx.x & 63) == 0 && __ballot(any) != 0ull) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            atomicMin(&bounds[k], mn[k]);
            atomicMax(&bounds[3 + k], mx[k]);
        }
    }
}

// box of all finite segment endpoints (the clip box of the chunked lines)
__global__ __launch_bounds__(kBlock) void k_seg_bounds(int64_t nseg, const float *__restrict__ o,
                                                       const float *__restrict__ p, unsigned int *__restrict__ bounds) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    unsigned int mn[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, mx[3] = {0u, 0u, 0u};
    bool any = false;
    if (i < nseg) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const float *q = (e == 0 ? o : p) + 3 * i;
            const float v[3] = {q[0], q[1], q[2]};
            if (isfinite(v[0]) && isfinite(v[1]) && isfinite(v[2])) {
                any = true;
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    mn[k] = min(mn[k], f2ord(v[k]));
                    mx[k] = max(mx[k], f2ord(v[k]));
                }
            }
        }
    }
    wave_minmax_atomic(mn, mx, any, bounds);
}

struct Clip {
    f3 lo, hi;
    float margin;  // absolute rounding margin ~1e-5 of the scene scale
};
__device__ __forceinline__ Clip load_clip(const unsigned int *b) {
    Clip c;
    c.lo = mk(ord2f(b[0]), ord2f(b[1]), ord2f(b[2]));
    c.hi = mk(ord2f(b[3]), ord2f(b[4]), ord2f(b[5]));
    const float m = fmaxf(fmaxf(fmaxf(fabsf(c.lo.x), fabsf(c.lo.y)), fmaxf(fabsf(c.lo.z), fabsf(c.hi.x))),
                          fmaxf(fabsf(c.hi.y), fabsf(c.hi.z)));
    c.margin = 1e-5f * (1.0f + m);
    return c;
}

__device__ __forceinline__ float chunk_E(float R, float r, float margin) { return (R + r) * 1.001f + margin; }

// Parameter interval of the line b0 + bu*s inside [lo, hi]; false when it misses.
__device__ __forceinline__ bool clip_line(f3 b0, f3 bu, f3 lo, f3 hi, float &t_in, float &t_out) {
    float a = -FLT_MAX, b = FLT_MAX;
    const float o[3] = {b0.x, b0.y, b0.z}, d[3] = {bu.x, bu.y, bu.z};
    const float l[3] = {lo.x, lo.y, lo.z}, h[3] = {hi.x, hi.y, hi.z};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        if (d[k] == 0.f) {
            if (o[k] < l[k] || o[k] > h[k]) return false;
        } else {
            float t0 = (l[k] - o[k]) / d[k], t1 = (h[k] - o[k]) / d[k];
            if (t0 > t1) {
                const float x = t0;
                t0 = t1;
                t1 = x;
            }
            a = fmaxf(a, t0);
            b = fminf(b, t1);
        }
    }
    t_in = a;
    t_out = b;
    return a <= b;
}

__device__ __forceinline__ bool parent_usable(const BeamRec &r) {
    // a NaN / infinite reference box is never hit (so the beam never contributes); a zero-length
    // beam has one (photonbeambvh.h:60-72: dir / 0)
    bool ok = r.mag_b > 0.f && isfinite(r.mag_b);
#pragma unroll
    for (int k = 0; k < 3; ++k)
        ok = ok && isfinite(r.lo[k]) && isfinite(r.hi[k]) && isfinite(r.b0[k]) && isfinite(r.bu[k]);
    return ok;
}

__global__ __launch_bounds__(kBlock) void k_chunk_count(const BeamRec *__restrict__ parents, BeamSet bset, int64_t n,
                                                        const unsigned int *__restrict__ seg_bounds, float R,
                                                        float len_factor, int32_t *__restrict__ counts,
                                                        float *__restrict__ range) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const BeamRec r = parents[i];
    int cnt = 0;
    float t_in = 0.f, t_out = 0.f;
    if (parent_usable(r) && seg_bounds[0] <= seg_bounds[3]) {
        const Clip c = load_clip(seg_bounds);
        const float E = chunk_E(R, beam_radius(bset, r.radius), c.margin);
        const f3 lo = mk(c.lo.x - E, c.lo.y - E, c.lo.z - E), hi = mk(c.hi.x + E, c.hi.y + E, c.hi.z + E);
        const f3 b0 = mk(r.b0[0], r.b0[1], r.b0[2]), bu = mk(r.bu[0], r.bu[1], r.bu[2]);
        if (isfinite(E) && E > 0.f && clip_line(b0, bu, lo, hi, t_in, t_out)) {
            const float len = fmaxf(t_out - t_in, 0.f);
            const float ell = len_factor * E;
            cnt = (int)fminf(ceilf(len / ell), (float)kMaxChunksPerBeam);
            cnt = cnt < 1 ? 1 : cnt;
        }
    }
    counts[i] = cnt;
    range[2 * i] = t_in;
    range[2 * i + 1] = t_out;
}

__global__ __launch_bounds__(kBlock) void k_chunk_emit(const BeamRec *__restrict__ parents, BeamSet bset, int64_t n,
                                                       const unsigned int *__restrict__ seg_bounds, float R,
                                                       const int32_t *__restrict__ counts,
                                                       const int64_t *__restrict__ offsets,
                                                       const float *__restrict__ range, float *__restrict__ box,
                                                       float *__restrict__ cent, float *__restrict__ s_lo,
                                                       float *__restrict__ s_hi, int32_t *__restrict__ parent,
                                                       unsigned int *__restrict__ cbounds) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    unsigned int mn[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, mx[3] = {0u, 0u, 0u};
    const int cnt = i < n ? counts[i] : 0;
    if (cnt > 0) {
        const BeamRec r = parents[i];
        const Clip c = load_clip(seg_bounds);
        const float E = chunk_E(R, beam_radius(bset, r.radius), c.margin);
        const f3 b0 = mk(r.b0[0], r.b0[1], r.b0[2]), bu = mk(r.bu[0], r.bu[1], r.bu[2]);
        const float t_in = range[2 * i], t_out = range[2 * i + 1];
        const float span = t_out - t_in, fn = (float)cnt;
        const int64_t w = offsets[i];
        for (int k = 0; k < cnt; ++k) {
            // the boundary between chunks k and k+1 is the same float expression in both
            const float a = t_in + span * ((float)k / fn);
            const float b = (k + 1 == cnt) ? t_out : t_in + span * ((float)(k + 1) / fn);
            const f3 p0 = add3(b0, scale3(bu, a)), p1 = add3(b0, scale3(bu, b));
            const float bx[6] = {fminf(p0.x, p1.x) - E, fminf(p0.y, p1.y) - E, fminf(p0.z, p1.z) - E,
                                 fmaxf(p0.x, p1.x) + E, fmaxf(p0.y, p1.y) + E, fmaxf(p0.z, p1.z) + E};
            const int64_t j = w + k;
#pragma unroll
            for (int q = 0; q < 6; ++q) box[6 * j + q] = bx[q];
            const float cc[3] = {0.5f * (bx[0] + bx[3]), 0.5f * (bx[1] + bx[4]), 0.5f * (bx[2] + bx[5])};
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                cent[3 * j + q] = cc[q];
                mn[q] = min(mn[q], f2ord(cc[q]));
                mx[q] = max(mx[q], f2ord(cc[q]));
            }
            s_lo[j] = (k == 0) ? -__builtin_huge_valf() : a;
            s_hi[j] = (k + 1 == cnt) ? __builtin_huge_valf() : b;
            parent[j] = (int32_t)i;
        }
    }
    wave_minmax_atomic(mn, mx, cnt > 0, cbounds);
}

__global__ __launch_bounds__(kBlock) void k_chunk_pack(const BeamRec *__restrict__ parents, BeamSet bset,
                                                       int64_t nchunks,
                                                       const int32_t *__restrict__ order,
                                                       const float *__restrict__ box, const float *__restrict__ s_lo,
                                                       const float *__restrict__ s_hi,
                                                       const int32_t *__restrict__ parent, ChunkRec *__restrict__ out,
                                                       int32_t *__restrict__ out_parent) {
    const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= nchunks) return;
    const int32_t c = order[j];
    const int32_t pi = parent[c];
    const BeamRec r = parents[pi];
    ChunkRec q;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        q.lo[k] = box[6 * (int64_t)c + k];
        q.hi[k] = box[6 * (int64_t)c + 3 + k];
        q.b0[k] = r.b0[k];
        q.bu[k] = r.bu[k];
    }
    q.mag_b = r.mag_b;
    q.radius = beam_radius(bset, r.radius);
    q.s_lo = s_lo[c];
    q.s_hi = s_hi[c];
    out[j] = q;
    out_parent[j] = pi;
}

// ---------------------------------------------------------------------------------------------
// Gather: thread-per-segment traversal of the chunk LBVH (per-thread stack in LDS).
struct ChunkV {
    Box6 box;
    f3 b0, bu;
    float mag_b, radius, s_lo, s_hi;
};
__device__ __forceinline__ ChunkV load_chunk(const ChunkRec *__restrict__ recs, int64_t i) {
    const float4 *q = reinterpret_cast<const float4 *>(recs + i);
    const float4 x = q[0], y = q[1], z = q[2], w = q[3];
    ChunkV r;
    r.box = Box6{x.x, x.y, x.z, x.w, y.x, y.y};
    r.b0 = mk(y.z, y.w, z.x);
    r.bu = mk(z.y, z.z, z.w);
    r.mag_b = w.x;
    r.radius = w.y;
    r.s_lo = w.z;
    r.s_hi = w.w;
    return r;
}

struct ChunkAcc {
    float r = 0.f, g = 0.f, b = 0.f;
    int ccp = 0, contrib = 0;
};

template <bool COUNT, bool PREF>
__device__ __forceinline__ void eval_chunk(const Lane &L, const ChunkV &c, int64_t j, float R,
                                           const int32_t *__restrict__ cpar, const BeamRec *__restrict__ parents,
                                           const float4 *__restrict__ pw, ChunkAcc &acc) {
    const float maxd = R + c.radius;  // MaxDistance = currentBeamRadius + beam->radius
    if (PREF && far_from_lines_fast(L.o, L.au, L.mag_a, L.omax, c.b0, c.bu, maxd)) return;
    float dist, s;
    const bool ok = closest_distance_t<true>(L.o, L.p, L.au, L.mag_a, c.b0, c.bu, c.mag_b, dist, s);
    if (COUNT) acc.ccp += ok;
    if (!(ok & (dist < maxd) & (s >= c.s_lo) & (s < c.s_hi))) return;
    // the reference's candidate test on the parent's (group) box, exactly as kernels 1-4
    const int32_t pi = cpar[j];
    const BeamRec *pr = parents + pi;
    const float4 *q = reinterpret_cast<const float4 *>(pr);
    const float4 x = q[0], y = q[1];
    const Box6 pb{x.x, x.y, x.z, x.w, y.x, y.y};
    float te;
    const bool hit = L.has_inf ? slab_test(pb, L.o, L.inv, L.n0, L.n1, L.n2, L.tmax, nullptr)
                               : node_test(pb, L.o, L.invs, L.tmax, te);
    if (!hit) return;
    const float rr = dist / maxd;
    const float wgt = sqrtf(1.0f - rr * rr);
    const float4 pv = pw[pi];
    acc.r += pv.x * wgt;
    acc.g += pv.y * wgt;
    acc.b += pv.z * wgt;
    ++acc.contrib;  // always: seg_counts[1] is defined without counters too (C = -1 then)
}

template <bool COUNT, bool PREF>
__global__ __launch_bounds__(kChunkBlock) void k_gather_chunk(
    int64_t nseg, const float *__restrict__ so, const float *__restrict__ sp_, const float *__restrict__ sd,
    const float *__restrict__ stmax, const int32_t *__restrict__ pixel, float R, int64_t npix,
    float *__restrict__ accum, float *__restrict__ seg_rgb, int32_t *__restrict__ seg_counts,
    const ChunkRec *__restrict__ recs, const int32_t *__restrict__ cpar, const BeamRec *__restrict__ parents,
    const float4 *__restrict__ pw, const Node *__restrict__ nodes, int64_t nchunks, int leaf_size,
    DevCounters *ctr) {
    __shared__ int32_t stk[kChunkStack][kChunkBlock];
    const int tid = threadIdx.x;
    const int64_t s = (int64_t)blockIdx.x * kChunkBlock + tid;
    Lane L;
    const bool valid = load_lane(s, nseg, so, sp_, sd, stmax, L);
    // traversal ray: the whole segment plus a rounding margin (chunk boxes are conservative)
    const float tq = L.tmax * 1.0001f + 1e-6f;
    ChunkAcc acc;
    unsigned long long visits = 0;
    if (valid && nchunks > 0) {
        int node = 0;
        int sp = 0;
        if (nchunks == 1) {
            eval_chunk<COUNT, PREF>(L, load_chunk(recs, 0), 0, R, cpar, parents, pw, acc);
        } else {
            while (true) {
                const NodeV n = load_node(nodes, node);
                if (COUNT) ++visits;
                const int32_t c0 = n.c0, c1 = n.c1;
                float te0 = 0.f, te1 = 0.f;
                bool h0 = (c0 != kEmptyChild) & node_test(n.b0, L.o, L.invs, tq, te0);
                bool h1 = (c1 != kEmptyChild) & node_test(n.b1, L.o, L.invs, tq, te1);
                if (h0 && c0 < 0) {
                    const int64_t first = (int64_t)(~c0) * leaf_size;
                    const int cnt = (int)min((int64_t)leaf_size, nchunks - first);
                    for (int j = 0; j < cnt; ++j) {
                        const ChunkV cv = load_chunk(recs, first + j);
                        float te;
                        if (leaf_size == 1 || node_test(cv.box, L.o, L.invs, tq, te))
                            eval_chunk<COUNT, PREF>(L, cv, first + j, R, cpar, parents, pw, acc);
                    }
                    h0 = false;
                }
                if (h1 && c1 < 0) {
                    const int64_t first = (int64_t)(~c1) * leaf_size;
                    const int cnt = (int)min((int64_t)leaf_size, nchunks - first);
                    for (int j = 0; j < cnt; ++j) {
                        const ChunkV cv = load_chunk(recs, first + j);
                        float te;
                        if (leaf_size == 1 || node_test(cv.box, L.o, L.invs, tq, te))
                            eval_chunk<COUNT, PREF>(L, cv, first + j, R, cpar, parents, pw, acc);
                    }
                    h1 = false;
                }
                if (h0 && h1) {
                    const bool first0 = !(te1 < te0);
                    if (sp >= kChunkStack) {
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
    }
    if (valid) {
        if (seg_rgb) {
            seg_rgb[3 * s] = acc.r;
            seg_rgb[3 * s + 1] = acc.g;
            seg_rgb[3 * s + 2] = acc.b;
        }
        if (accum) {
            const int32_t px = pixel[s];
            if (px < 0 || px >= npix) {
                atomicOr(&ctr->flags, kFlagPixel);
            } else if (acc.r != 0.f || acc.g != 0.f || acc.b != 0.f) {
                atomicAdd(&accum[3 * (int64_t)px], acc.r);
                atomicAdd(&accum[3 * (int64_t)px + 1], acc.g);
                atomicAdd(&accum[3 * (int64_t)px + 2], acc.b);
            }
        }
        if (seg_counts) {
            seg_counts[2 * s] = COUNT ? acc.ccp : -1;
            seg_counts[2 * s + 1] = acc.contrib;
        }
    }
    if (COUNT) {
        unsigned long long c = valid ? (unsigned long long)acc.ccp : 0ull;
        unsigned long long k = valid ? (unsigned long long)acc.contrib : 0ull;
        unsigned long long v = visits;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            c += __shfl_xor(c, off);
            k += __shfl_xor(k, off);
            v += __shfl_xor(v, off);
        }
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(&ctr->ccp_wave_evals, c);
            atomicAdd(&ctr->contributions, k);
            atomicAdd(&ctr->node_visits, v);
        }
    }
}

__global__ void k_init_bounds(unsigned int *a, unsigned int *b) {
    const int t = threadIdx.x;
    if (t < 6) {
        a[t] = t < 3 ? 0xffffffffu : 0u;
        b[t] = t < 3 ? 0xffffffffu : 0u;
    }
}

inline unsigned grid_of(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

}  // namespace

size_t chunk_scan_temp_bytes(int64_t n) {
    size_t bytes = 0;
    (void)rocprim::inclusive_scan(nullptr, bytes, (const int32_t *)nullptr, (int64_t *)nullptr, (size_t)n,
                                  rocprim::plus<int64_t>());
    return bytes;
}

hipError_t launch_chunk_count(const ChunkBuild &c, hipStream_t s) {
    hipLaunchKernelGGL(k_init_bounds, dim3(1), dim3(64), 0, s, c.seg_bounds, c.cbounds);
    if (c.nseg > 0)
        hipLaunchKernelGGL(k_seg_bounds, dim3(grid_of(c.nseg, kBlock)), dim3(kBlock), 0, s, c.nseg, c.seg_o, c.seg_p,
                           c.seg_bounds);
    if (c.nparents > 0)
        hipLaunchKernelGGL(k_chunk_count, dim3(grid_of(c.nparents, kBlock)), dim3(kBlock), 0, s, c.parents,
                           c.bset, c.nparents, c.seg_bounds, c.R, c.len_factor, c.counts, c.range);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(c.offsets, 0, sizeof(int64_t), s);
    if (e != hipSuccess || c.nparents == 0) return e;
    size_t bytes = c.scan_tmp_bytes;
    return rocprim::inclusive_scan(c.scan_tmp, bytes, (const int32_t *)c.counts, c.offsets + 1, (size_t)c.nparents,
                                   rocprim::plus<int64_t>(), s);
}

hipError_t launch_chunk_emit(const ChunkBuild &c, float *box, float *cent, float *s_lo, float *s_hi,
                             int32_t *parent, hipStream_t s) {
    if (c.nparents == 0) return hipSuccess;
    hipLaunchKernelGGL(k_chunk_emit, dim3(grid_of(c.nparents, kBlock)), dim3(kBlock), 0, s, c.parents, c.bset,
                       c.nparents, c.seg_bounds, c.R, c.counts, c.offsets, c.range, box, cent, s_lo, s_hi, parent, c.cbounds);
    return hipGetLastError();
}

hipError_t launch_chunk_pack(const ChunkBuild &c, int64_t nchunks, const int32_t *order, const float *box,
                             const float *s_lo, const float *s_hi, const int32_t *parent, ChunkRec *out,
                             int32_t *out_parent, hipStream_t s) {
    if (nchunks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_chunk_pack, dim3(grid_of(nchunks, kBlock)), dim3(kBlock), 0, s, c.parents, c.bset, nchunks,
                       order,
                       box, s_lo, s_hi, parent, out, out_parent);
    return hipGetLastError();
}

hipError_t launch_gather_chunk(const ChunkGatherArgs &a, bool counters, hipStream_t s) {
    if (a.nseg == 0) return hipSuccess;
    const dim3 grid(grid_of(a.nseg, kChunkBlock));
#define BRE_LAUNCH_CHUNK(C, P)                                                                                     \
    hipLaunchKernelGGL((k_gather_chunk<C, P>), grid, dim3(kChunkBlock), 0, s, a.nseg, a.o, a.p, a.d, a.tmax,       \
                       a.pixel, a.R, a.npix, a.accum, a.seg_rgb, a.seg_counts, a.chunks, a.chunk_parent, a.parents, \
                       a.pow, a.nodes, a.nchunks, a.leaf_size, a.ctr)
    if (counters) {
        if (a.prefilter) BRE_LAUNCH_CHUNK(true, true);
        else BRE_LAUNCH_CHUNK(true, false);
    } else {
        if (a.prefilter) BRE_LAUNCH_CHUNK(false, true);
        else BRE_LAUNCH_CHUNK(false, false);
    }
#undef BRE_LAUNCH_CHUNK
    return hipGetLastError();
}

}  // namespace bre
