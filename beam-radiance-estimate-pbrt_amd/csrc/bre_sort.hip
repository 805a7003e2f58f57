// bre_sort.hip — coherence sort of an iteration's camera segments before the gather.
//
// The reference gathers segment by segment inside each camera path (photonbeam.cpp:494-508); the
// batched gather is order-free (each segment's sum goes to its pixel), so the segments can be
// handed to the packet kernels in any order.  Camera rays of one 8x8 pixel tile form coherent
// 64-lane packets, but the bounce segments (depth >= 1) leave the walls in cosine-distributed
// directions: a packet of 64 unrelated rays visits the union of 64 traversals.  Sorting by a 5-D
// Morton key of (origin in the segments' box, octahedral direction) puts segments that start
// close together AND point the same way into the same packet, so the packet kernels share most
// of their node and beam visits again.  The default key (mode 1) interleaves the segment's origin
// and end point instead (6-D Morton): two segments with both ends close are close all along, which
// at C2 shortens the gather by ~5% over the (origin, direction) key (mode 0).  Only the order changes; every per-segment sum and every
// pixel total is the same set of pair contributions.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <rocprim/device/device_radix_sort.hpp>

#include <float.h>

#include "bre_device.h"
#include "bre_math.h"

namespace bre {

namespace {

#ifndef BRE_PASS_BLOCK
#define BRE_PASS_BLOCK 64  // one wave (bre_slot.hip; 256 until round 5)
#endif
constexpr int kBlock = BRE_PASS_BLOCK;  // threads per block of the pass kernels

__device__ __forceinline__ unsigned int f2ord(float f) {
    unsigned int u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(unsigned int u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

__global__ void k_sort_init(unsigned int *b) {
    if (threadIdx.x < 6) b[threadIdx.x] = threadIdx.x < 3 ? 0xffffffffu : 0u;
}

__global__ __launch_bounds__(kBlock) void k_origin_bounds(int64_t n, const float *__restrict__ o,
                                                          unsigned int *__restrict__ b) {
    // (key mode 1 launches it twice, over the origins and the end points, into one box).
    // Grid-stride with a block reduction: one set of 6 atomics per block, not per wave.
    __shared__ unsigned int red[kBlock / 64][6];
    unsigned int mn[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, mx[3] = {0u, 0u, 0u};
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        const float v[3] = {o[3 * i], o[3 * i + 1], o[3 * i + 2]};
        if (isfinite(v[0]) && isfinite(v[1]) && isfinite(v[2])) {
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                mn[k] = min(mn[k], f2ord(v[k]));
                mx[k] = max(mx[k], f2ord(v[k]));
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
    if (threadIdx.x == 0) {
        for (int v = 1; v < kBlock / 64; ++v) {
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                mn[k] = min(mn[k], red[v][k]);
                mx[k] = max(mx[k], red[v][3 + k]);
            }
        }
        if (mn[0] <= mx[0]) {  // at least one finite point
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                atomicMin(&b[k], mn[k]);
                atomicMax(&b[3 + k], mx[k]);
            }
        }
    }
}

__device__ __forceinline__ unsigned int quant10(float x) {  // x in [0, 1]
    const float q = fminf(fmaxf(x, 0.f), 1.f) * 1023.f;
    return (unsigned int)q;
}

// 5-D Morton key: 10 bits each of origin x, y, z (in the origins' box) and the octahedral
// direction u, v, interleaved from the most significant bit down
__global__ __launch_bounds__(kBlock) void k_seg_keys(int64_t n, const float *__restrict__ o,
                                                     const float *__restrict__ d, const unsigned int *__restrict__ b,
                                                     unsigned long long *__restrict__ keys,
                                                     int32_t *__restrict__ vals) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const float lo[3] = {ord2f(b[0]), ord2f(b[1]), ord2f(b[2])};
    const float hi[3] = {ord2f(b[3]), ord2f(b[4]), ord2f(b[5])};
    unsigned int q[5];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float ext = hi[k] - lo[k];
        q[k] = quant10(ext > 0.f ? (o[3 * i + k] - lo[k]) / ext : 0.f);
    }
    // octahedral map of the direction
    float dx = d[3 * i], dy = d[3 * i + 1], dz = d[3 * i + 2];
    const float l1 = fabsf(dx) + fabsf(dy) + fabsf(dz);
    float u = 0.f, v = 0.f;
    if (l1 > 0.f && isfinite(l1)) {
        dx /= l1;
        dy /= l1;
        dz /= l1;
        u = dx;
        v = dy;
        if (dz < 0.f) {
            u = (1.f - fabsf(dy)) * (dx >= 0.f ? 1.f : -1.f);
            v = (1.f - fabsf(dx)) * (dy >= 0.f ? 1.f : -1.f);
        }
    }
    q[3] = quant10(0.5f * u + 0.5f);
    q[4] = quant10(0.5f * v + 0.5f);
    unsigned long long key = 0ull;
#pragma unroll
    for (int bit = 9; bit >= 0; --bit)
#pragma unroll
        for (int k = 0; k < 5; ++k) key = (key << 1) | ((q[k] >> bit) & 1u);
    keys[i] = key;
    vals[i] = (int32_t)i;
}

// 6-D Morton key: 10 bits each of origin x, y, z and end point x, y, z (in the box of both)
__global__ __launch_bounds__(kBlock) void k_seg_keys_op(int64_t n, const float *__restrict__ o,
                                                        const float *__restrict__ p, const unsigned int *__restrict__ b,
                                                        int hilbert, unsigned long long *__restrict__ keys,
                                                        int32_t *__restrict__ vals) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const float lo[3] = {ord2f(b[0]), ord2f(b[1]), ord2f(b[2])};
    const float hi[3] = {ord2f(b[3]), ord2f(b[4]), ord2f(b[5])};
    unsigned int q[6];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float ext = hi[k] - lo[k];
        q[k] = quant10(ext > 0.f ? (o[3 * i + k] - lo[k]) / ext : 0.f);
        q[3 + k] = quant10(ext > 0.f ? (p[3 * i + k] - lo[k]) / ext : 0.f);
    }
    unsigned long long key = 0ull;
    if (hilbert) {
        key = hilbert_key<6, 10>(q);
    } else {
#pragma unroll
        for (int bit = 9; bit >= 0; --bit)
#pragma unroll
            for (int k = 0; k < 6; ++k) key = (key << 1) | ((q[k] >> bit) & 1u);
    }
    keys[i] = key;
    vals[i] = (int32_t)i;
}

// Line keys (modes 2 / 3): the packet kernels' bundle reject measures how far the packet's segments
// lie from ONE line, so segments on nearly the same infinite line belong together wherever they sit
// along it.  The key is the segment's line: a class of 3 bits for the dominant axis a of its
// direction and that component's sign, then Morton bits of the two slopes dir_b / |dir_a|,
// dir_c / |dir_a| (in [-1, 1]) and of the point where the line crosses the plane x_a = centre_a of
// the segments' box (the other two coordinates, in the box grown by its extent on both sides).
// Mode 2 interleaves these 4 coordinates with 14 bits each; mode 3 adds the segment midpoint's
// coordinate along the dominant axis as a fifth, with 11 bits each.
__device__ __forceinline__ unsigned int quant_bits(float x, int bits) {  // x in [0, 1]
    const float m = (float)((1u << bits) - 1u);
    return (unsigned int)(fminf(fmaxf(x, 0.f), 1.f) * m);
}

__global__ __launch_bounds__(kBlock) void k_seg_keys_line(int64_t n, const float *__restrict__ o,
                                                          const float *__restrict__ p, const float *__restrict__ d,
                                                          const unsigned int *__restrict__ b, int five,
                                                          unsigned long long *__restrict__ keys,
                                                          int32_t *__restrict__ vals) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const float lo[3] = {ord2f(b[0]), ord2f(b[1]), ord2f(b[2])};
    const float hi[3] = {ord2f(b[3]), ord2f(b[4]), ord2f(b[5])};
    const float O[3] = {o[3 * i], o[3 * i + 1], o[3 * i + 2]};
    const float P[3] = {p[3 * i], p[3 * i + 1], p[3 * i + 2]};
    float v[3] = {P[0] - O[0], P[1] - O[1], P[2] - O[2]};
    if (!(fabsf(v[0]) + fabsf(v[1]) + fabsf(v[2]) > 0.f)) {  // zero-length segment: its ray direction
        v[0] = d[3 * i];
        v[1] = d[3 * i + 1];
        v[2] = d[3 * i + 2];
    }
    int a = 0;
    if (fabsf(v[1]) > fabsf(v[a])) a = 1;
    if (fabsf(v[2]) > fabsf(v[a])) a = 2;
    const int b1 = a == 0 ? 1 : 0, b2 = a == 2 ? 1 : 2;
    const float va = v[a];
    const unsigned int cls = (unsigned int)(2 * a + (va < 0.f ? 1 : 0));
    const float ia = va != 0.f && isfinite(va) ? 1.f / fabsf(va) : 0.f;
    float q[5];
    q[0] = 0.5f * (v[b1] * ia) + 0.5f;  // slopes in [-1, 1] -> [0, 1]
    q[1] = 0.5f * (v[b2] * ia) + 0.5f;
    const float ca = 0.5f * (lo[a] + hi[a]);
    const float t = va != 0.f ? (ca - O[a]) / va : 0.f;
    const int bb[2] = {b1, b2};
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int c = bb[k];
        const float ext = hi[c] - lo[c];
        const float x = O[c] + t * v[c];
        q[2 + k] = ext > 0.f ? (x - (lo[c] - ext)) / (3.f * ext) : 0.f;
    }
    {
        const float ext = hi[a] - lo[a];
        q[4] = ext > 0.f ? (0.5f * (O[a] + P[a]) - lo[a]) / ext : 0.f;
    }
    unsigned long long key = cls;
    if (five) {
        unsigned int u[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) u[k] = quant_bits(isfinite(q[k]) ? q[k] : 0.f, 11);
#pragma unroll
        for (int bit = 10; bit >= 0; --bit)
#pragma unroll
            for (int k = 0; k < 5; ++k) key = (key << 1) | ((u[k] >> bit) & 1u);
    } else {
        unsigned int u[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) u[k] = quant_bits(isfinite(q[k]) ? q[k] : 0.f, 14);
#pragma unroll
        for (int bit = 13; bit >= 0; --bit)
#pragma unroll
            for (int k = 0; k < 4; ++k) key = (key << 1) | ((u[k] >> bit) & 1u);
    }
    keys[i] = key;
    vals[i] = (int32_t)i;
}

__global__ __launch_bounds__(kBlock) void k_seg_permute(int64_t n, const int32_t *__restrict__ order,
                                                        const float *__restrict__ o, const float *__restrict__ p,
                                                        const float *__restrict__ d, const float *__restrict__ t,
                                                        const int32_t *__restrict__ pix, float *__restrict__ o2,
                                                        float *__restrict__ p2, float *__restrict__ d2,
                                                        float *__restrict__ t2, int32_t *__restrict__ pix2) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const int64_t j = order[i];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        o2[3 * i + k] = o[3 * j + k];
        p2[3 * i + k] = p[3 * j + k];
        d2[3 * i + k] = d[3 * j + k];
    }
    t2[i] = t[j];
    pix2[i] = pix ? pix[j] : 0;  // no pixel array: a gather without a film (per-segment outputs only)
}

inline unsigned grid_of(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

// Packet shards: copy this shard's packets into contiguous arrays -- the sorted order's 64-segment
// packets in chunks of `chunk` consecutive packets, chunk c to shard c mod count (bre_shard_segments);
// index2 (optional) carries the source's caller index.
__global__ __launch_bounds__(kBlock) void k_packet_pick(int64_t n, int64_t m, int rank, int count, int chunk,
                                                        const float *__restrict__ o, const float *__restrict__ p,
                                                        const float *__restrict__ d, const float *__restrict__ t,
                                                        const int32_t *__restrict__ pix,
                                                        const int32_t *__restrict__ index, float *__restrict__ o2,
                                                        float *__restrict__ p2, float *__restrict__ d2,
                                                        float *__restrict__ t2, int32_t *__restrict__ pix2,
                                                        int32_t *__restrict__ index2) {
    const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= m) return;
    const int64_t g = j >> 6;  // this shard's packet ordinal: chunk g / chunk, packet g % chunk in it
    const int64_t src = (((g / chunk) * count + rank) * chunk + g % chunk) * 64 + (j & 63);  // < n for j < m
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        o2[3 * j + k] = o[3 * src + k];
        p2[3 * j + k] = p[3 * src + k];
        d2[3 * j + k] = d[3 * src + k];
    }
    t2[j] = t[src];
    pix2[j] = pix ? pix[src] : 0;
    if (index2) index2[j] = index ? index[src] : (int32_t)src;
    (void)n;
}

// Deterministic per-pixel accumulation of a gather's per-segment sums (PixelCompose).  The reference
// adds a pixel's gather terms in one fixed order (one thread per 16x16 tile, the pixel's path depths
// in order, photonbeam.cpp:477-504); float atomics would add a pixel's segments in arrival order and
// let the film differ in the last bits from run to run.  Instead the segments are stably sorted by
// pixel (so a pixel's segments keep the caller's order: the camera pass's depth order), and one
// thread per pixel adds its run of segment sums in that order and then adds the run's sum to the film.
// With film classes (BRE_OPT_FILM_CLASSES) the key is class * (npix + 1) + pixel: a class's pixels in
// order, each class's slot npix marking an invalid pixel.
__global__ __launch_bounds__(kBlock) void k_pix_keys(int64_t n, const int32_t *__restrict__ pix, int64_t npix,
                                                     const uint8_t *__restrict__ cls,
                                                     unsigned int *__restrict__ keys, int32_t *__restrict__ vals) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const int32_t p = pix[i];
    const unsigned int base = cls ? (unsigned int)cls[i] * (unsigned int)(npix + 1) : 0u;
    keys[i] = base + ((p < 0 || (int64_t)p >= npix) ? (unsigned int)npix : (unsigned int)p);  // npix: invalid
    vals[i] = (int32_t)i;
}

__global__ __launch_bounds__(kBlock) void k_pix_compose(int64_t n, const unsigned int *__restrict__ keys,
                                                        const int32_t *__restrict__ vals,
                                                        const float *__restrict__ seg_rgb, int64_t npix,
                                                        float *__restrict__ accum, unsigned int *__restrict__ flags,
                                                        unsigned int bad_pixel_flag) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const unsigned int k = keys[i];
    if (i > 0 && keys[i - 1] == k) return;  // not the first segment of its pixel
    const int64_t cl = (int64_t)k / (npix + 1), px = (int64_t)k - cl * (npix + 1);
    if (px >= npix) {
        atomicOr(flags, bad_pixel_flag);  // a seg_pixel outside [0, npix): never silent (check_flags)
        return;
    }
    float r = 0.f, g = 0.f, b = 0.f;
    for (int64_t j = i; j < n && keys[j] == k; ++j) {
        const int64_t s = vals[j];
        r += seg_rgb[3 * s];
        g += seg_rgb[3 * s + 1];
        b += seg_rgb[3 * s + 2];
    }
    if (r != 0.f || g != 0.f || b != 0.f) {
        float *a = accum + 3 * (cl * npix + px);
        a[0] += r;
        a[1] += g;
        a[2] += b;
    }
}

// The film class of each segment (BRE_OPT_FILM_CLASSES): sorted segment i lies in packet chunk
// (i / 64) / block -- the unit bre_shard_segments deals to the shards -- and its class is that chunk
// mod `classes`, written at the segment's caller index.
__global__ __launch_bounds__(kBlock) void k_seg_classes(int64_t n, int block, int classes,
                                                        const int32_t *__restrict__ perm, uint8_t *__restrict__ cls) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const int64_t s = perm ? (int64_t)perm[i] : i;
    cls[s] = (uint8_t)(((i >> 6) / block) % classes);
}

// The image of the class films, added in class order (bit-identical wherever the planes are).  `out` may
// alias plane 0 of `in` (include/bre.h), so neither pointer is __restrict__: each thread reads its element
// of every plane before it stores out[i].
__global__ __launch_bounds__(kBlock) void k_resolve_classes(int64_t m, int classes, const float *in, float *out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= m) return;
    float v = in[i];
    for (int c = 1; c < classes; ++c) v += in[(int64_t)c * m + i];
    out[i] = v;
}

// dst += src (element-wise, a film of one iteration into the render's film), then src = 0 when asked
__global__ __launch_bounds__(kBlock) void k_film_add(int64_t m, float *src, float *__restrict__ dst, int clear) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < m; i += (int64_t)gridDim.x * kBlock) {
        dst[i] += src[i];
        if (clear) src[i] = 0.f;
    }
}

}  // namespace

hipError_t launch_film_add(int64_t m, float *src, float *dst, int clear, hipStream_t st) {
    if (m <= 0) return hipSuccess;
    const int64_t g = (m + 4 * kBlock - 1) / (4 * kBlock);
    hipLaunchKernelGGL(k_film_add, dim3((unsigned)std::min<int64_t>(g, 1 << 20)), dim3(kBlock), 0, st, m, src, dst, clear);
    return hipGetLastError();
}

hipError_t launch_seg_classes(int64_t n, int block, int classes, const int32_t *perm, uint8_t *cls, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_seg_classes, dim3(grid_of(n)), dim3(kBlock), 0, st, n, block < 1 ? 1 : block, classes, perm,
                       cls);
    return hipGetLastError();
}

hipError_t launch_resolve_classes(int64_t m, int classes, const float *in, float *out, hipStream_t st) {
    if (m <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_resolve_classes, dim3(grid_of(m)), dim3(kBlock), 0, st, m, classes, in, out);
    return hipGetLastError();
}

hipError_t launch_packet_pick(int64_t n, int64_t m, int rank, int count, int chunk, const float *o, const float *p,
                              const float *d, const float *t, const int32_t *pix, const int32_t *index, float *o2,
                              float *p2, float *d2, float *t2, int32_t *pix2, int32_t *index2, hipStream_t st) {
    if (m <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_packet_pick, dim3(grid_of(m)), dim3(kBlock), 0, st, n, m, rank, count, chunk, o, p, d, t, pix, index,
                       o2, p2, d2, t2, pix2, index2);
    return hipGetLastError();
}

size_t seg_sort_temp_bytes(int64_t n) {
    size_t bytes = 0;
    (void)rocprim::radix_sort_pairs(nullptr, bytes, (unsigned long long *)nullptr, (unsigned long long *)nullptr,
                                    (int32_t *)nullptr, (int32_t *)nullptr, (size_t)n, 0, 64);  // the widest key any mode sorts
    return std::max(bytes, slot_sort_temp_bytes(n, 8));
}

hipError_t launch_sort_segments(const SegSort &s, hipStream_t st) {
    if (s.n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_sort_init, dim3(1), dim3(64), 0, st, s.bounds);
    // grid-stride bounds over at most 256 blocks (one set of six same-address atomics per block)
    const unsigned bgrid = grid_of(s.n) < 256u ? grid_of(s.n) : 256u;
    hipLaunchKernelGGL(k_origin_bounds, dim3(bgrid), dim3(kBlock), 0, st, s.n, s.o, s.bounds);
    int key_bits = 50;
    if (s.key_mode == 1 || s.key_mode == 4) {
        hipLaunchKernelGGL(k_origin_bounds, dim3(bgrid), dim3(kBlock), 0, st, s.n, s.p, s.bounds);
        hipLaunchKernelGGL(k_seg_keys_op, dim3(grid_of(s.n)), dim3(kBlock), 0, st, s.n, s.o, s.p, s.bounds,
                           s.key_mode == 4 ? 1 : 0, s.keys, s.vals);
        key_bits = 60;
    } else if (s.key_mode == 2 || s.key_mode == 3) {
        hipLaunchKernelGGL(k_origin_bounds, dim3(bgrid), dim3(kBlock), 0, st, s.n, s.p, s.bounds);
        hipLaunchKernelGGL(k_seg_keys_line, dim3(grid_of(s.n)), dim3(kBlock), 0, st, s.n, s.o, s.p, s.d, s.bounds,
                           s.key_mode == 3 ? 1 : 0, s.keys, s.vals);
        key_bits = s.key_mode == 3 ? 58 : 59;
    } else {
        hipLaunchKernelGGL(k_seg_keys, dim3(grid_of(s.n)), dim3(kBlock), 0, st, s.n, s.o, s.d, s.bounds, s.keys,
                           s.vals);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    size_t bytes = s.tmp_bytes;
    const int lo = s.key_lo < key_bits ? s.key_lo : 0;
    e = s.slot ? slot_sort_pairs(s.tmp, s.keys, s.keys_alt, s.vals, s.vals_alt, s.n, lo, key_bits, st)
               : rocprim::radix_sort_pairs(s.tmp, bytes, s.keys, s.keys_alt, s.vals, s.vals_alt, (size_t)s.n,
                                           (unsigned int)lo, (unsigned int)key_bits, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_seg_permute, dim3(grid_of(s.n)), dim3(kBlock), 0, st, s.n, s.vals_alt, s.o, s.p, s.d, s.t,
                       s.pix, s.o2, s.p2, s.d2, s.t2, s.pix2);
    return hipGetLastError();
}

size_t pixel_sort_temp_bytes(int64_t n) {
    size_t bytes = 0;
    (void)rocprim::radix_sort_pairs(nullptr, bytes, (unsigned int *)nullptr, (unsigned int *)nullptr,
                                    (int32_t *)nullptr, (int32_t *)nullptr, (size_t)n, 0, 32);
    return std::max(bytes, slot_sort_temp_bytes(n, 4));
}

hipError_t launch_pixel_compose(const PixelCompose &c, hipStream_t st) {
    if (c.n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_pix_keys, dim3(grid_of(c.n)), dim3(kBlock), 0, st, c.n, c.pix, c.npix, c.cls, c.keys, c.vals);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const uint64_t top = (uint64_t)(c.cls ? c.classes : 1) * (uint64_t)(c.npix + 1);  // keys in [0, top)
    if (top > 0xffffffffull) return hipErrorInvalidValue;
    int bits = 1;
    while (bits < 32 && ((uint64_t)1 << bits) < top) ++bits;
    size_t bytes = c.tmp_bytes;
    e = c.slot ? slot_sort_pairs(c.tmp, c.keys, c.keys_alt, c.vals, c.vals_alt, c.n, 0, bits, st)
               : rocprim::radix_sort_pairs(c.tmp, bytes, c.keys, c.keys_alt, c.vals, c.vals_alt, (size_t)c.n, 0, bits, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_pix_compose, dim3(grid_of(c.n)), dim3(kBlock), 0, st, c.n, c.keys_alt, c.vals_alt, c.seg_rgb,
                       c.npix, c.accum, c.flags, c.bad_pixel_flag);
    return hipGetLastError();
}

}  // namespace bre
