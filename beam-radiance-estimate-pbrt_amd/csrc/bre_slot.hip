// bre_slot.hip — one-wave pass primitives: fill, exclusive scan and a stable LSD radix sort of
// (key, value) pairs, every kernel in 64-thread workgroups with at most 1 KB of LDS.
//
// Why (round 6, profiles/r6/e1): the pipelined render (bench.py --pipeline 1) runs iteration k+1's
// photon pass, BVH build, camera pass and segment sort on a high-priority stream while iteration k's
// gather occupies every CU with one-wave workgroups (80 VGPRs, 6 KB of LDS).  A retiring gather wave
// frees exactly one such slot, and the dispatcher fills it with the next gather wave unless a
// workgroup of the other queue fits it: a multi-wave workgroup, or one needing more LDS, waits until
// the gather's dispatch is over.  In the round-5 trace the photon kernel (two-wave workgroups) took
// 92 ms inside a 135 ms gather and the rest of the chain -- rocPRIM scans and sorts with 256- to
// 1024-thread workgroups and 11-33 KB of LDS, the runtime's memset and copy kernels, k_roots with
// 140 KB of LDS -- ran after it, 1.3-2.1 ms per iteration between the gathers.  With one-wave photon
// workgroups the photon pass took 5.6 ms inside the gather and the chain stalled at the next rocPRIM
// scan.  These primitives replace rocPRIM, hipMemsetAsync and the copy kernels on the pass chain so
// that every kernel of it fits a gather slot.  The sort is stable, so its permutation is rocPRIM's
// (radix_sort_pairs is stable too): every result is bit-identical.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "bre_device.h"

namespace bre {

namespace {

constexpr int kW = 64;            // one wave per workgroup
constexpr int kTileItems = 16;    // elements per lane per tile
constexpr int kTile = kW * kTileItems;  // 1024 elements per workgroup (scan and sort tiles)
constexpr int kMaxBins = 256;     // radix digits of at most 8 bits
constexpr unsigned kMaxGrid = 1u << 20;

inline unsigned tiles_of(int64_t n) { return (unsigned)((n + kTile - 1) / kTile); }
inline size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

__global__ __launch_bounds__(kW) void k_fill(unsigned int *__restrict__ p, int64_t n, unsigned int v) {
    for (int64_t i = (int64_t)blockIdx.x * kW + threadIdx.x; i < n; i += (int64_t)gridDim.x * kW) p[i] = v;
}

template <typename T>
__device__ __forceinline__ T wave_incl_scan(T v) {
    const int lane = threadIdx.x;
#pragma unroll
    for (int off = 1; off < kW; off <<= 1) {
        const T u = __shfl_up(v, off);
        if (lane >= off) v += u;
    }
    return v;
}

template <typename T>
__device__ __forceinline__ T wave_total(T v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// scan, step 1: the sum of each 1024-element tile
template <typename In, typename Out>
__global__ __launch_bounds__(kW) void k_scan_tile_sums(const In *__restrict__ in, int64_t n, Out *__restrict__ sums) {
    const int64_t base = (int64_t)blockIdx.x * kTile;
    Out s = 0;
#pragma unroll 4
    for (int r = 0; r < kTileItems; ++r) {
        const int64_t i = base + r * kW + threadIdx.x;
        if (i < n) s += (Out)in[i];
    }
    s = wave_total(s);
    if (threadIdx.x == 0) sums[blockIdx.x] = s;
}

// scan, step 2: one workgroup scans the tile sums in place (exclusive); *total (may be null) = the sum
template <typename Out>
__global__ __launch_bounds__(kW) void k_scan_sums(Out *__restrict__ sums, int64_t nt, Out *__restrict__ total) {
    Out carry = 0;
    for (int64_t b = 0; b < nt; b += kW) {
        const int64_t i = b + threadIdx.x;
        const Out v = i < nt ? sums[i] : (Out)0;
        const Out s = wave_incl_scan(v);
        if (i < nt) sums[i] = carry + s - v;
        carry += __shfl(s, kW - 1);
    }
    if (total && threadIdx.x == 0) *total = carry;
}

// scan, step 3: each tile's exclusive scan from its offset (out may be in)
template <typename In, typename Out>
__global__ __launch_bounds__(kW) void k_scan_tile(const In *in, int64_t n, const Out *__restrict__ sums, Out *out) {
    const int64_t base = (int64_t)blockIdx.x * kTile;
    Out carry = sums[blockIdx.x];
    for (int r = 0; r < kTileItems; ++r) {
        const int64_t i = base + r * kW + threadIdx.x;
        if (base + r * kW >= n) break;
        const Out v = i < n ? (Out)in[i] : (Out)0;
        const Out s = wave_incl_scan(v);
        if (i < n) out[i] = carry + s - v;
        carry += __shfl(s, kW - 1);
    }
}

template <typename In, typename Out>
hipError_t scan_impl(const In *in, Out *out, int64_t n, Out *total, void *tmp, hipStream_t s) {
    if (n <= 0) {
        if (total) hipLaunchKernelGGL(k_fill, dim3(1), dim3(kW), 0, s, reinterpret_cast<unsigned int *>(total),
                                      (int64_t)(sizeof(Out) / 4), 0u);
        return hipGetLastError();
    }
    const unsigned nt = tiles_of(n);
    Out *sums = static_cast<Out *>(tmp);
    hipLaunchKernelGGL((k_scan_tile_sums<In, Out>), dim3(nt), dim3(kW), 0, s, in, n, sums);
    hipLaunchKernelGGL((k_scan_sums<Out>), dim3(1), dim3(kW), 0, s, sums, (int64_t)nt, total);
    hipLaunchKernelGGL((k_scan_tile<In, Out>), dim3(nt), dim3(kW), 0, s, in, n, sums, out);
    return hipGetLastError();
}

// ---- stable LSD radix sort of (key, int32 value) pairs ----
// Per pass (a digit of db <= 8 bits): each 1024-element tile counts its digits (LDS atomics), the
// digit-major histogram (hist[d * nt + t]) is scanned into global offsets, and each tile scatters its
// elements in order -- an element's place is its tile's offset for its digit plus the number of
// same-digit elements before it in the tile (64 at a time: the lanes with an equal digit are the AND
// of db ballots, the lanes below it counted by mbcnt), so equal digits keep their order: stable.
template <typename K>
__global__ __launch_bounds__(kW) void k_digit_hist(const K *__restrict__ keys, int64_t n, int lo, int db,
                                                   int32_t *__restrict__ hist, int64_t nt) {
    __shared__ int32_t bins[kMaxBins];
    const int nb = 1 << db;
    for (int d = threadIdx.x; d < nb; d += kW) bins[d] = 0;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * kTile;
    const K mask = (K)(nb - 1);
#pragma unroll 4
    for (int r = 0; r < kTileItems; ++r) {
        const int64_t i = base + r * kW + threadIdx.x;
        if (i < n) atomicAdd(&bins[(int)((keys[i] >> lo) & mask)], 1);
    }
    __syncthreads();
    for (int d = threadIdx.x; d < nb; d += kW) hist[(int64_t)d * nt + blockIdx.x] = bins[d];
}

template <typename K>
__global__ __launch_bounds__(kW) void k_digit_scatter(const K *__restrict__ keys, const int32_t *__restrict__ vals,
                                                      int64_t n, int lo, int db, const int32_t *__restrict__ offs,
                                                      int64_t nt, K *__restrict__ keys_out,
                                                      int32_t *__restrict__ vals_out) {
    __shared__ int32_t run[kMaxBins];  // the next place of each digit in this tile
    const int nb = 1 << db;
    const int lane = threadIdx.x;
    for (int d = lane; d < nb; d += kW) run[d] = offs[(int64_t)d * nt + blockIdx.x];
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * kTile;
    const K mask = (K)(nb - 1);
    const unsigned long long below = (1ull << lane) - 1ull;
    for (int r = 0; r < kTileItems; ++r) {
        const int64_t i0 = base + r * kW;
        if (i0 >= n) break;
        const int64_t i = i0 + lane;
        const bool ok = i < n;
        const K k = ok ? keys[i] : (K)0;
        const int32_t v = ok ? vals[i] : 0;
        const int d = (int)((k >> lo) & mask);
        unsigned long long eq = __ballot(ok);
        for (int b = 0; b < db; ++b) {
            const bool bit = (d >> b) & 1;
            const unsigned long long m = __ballot(bit);
            eq &= bit ? m : ~m;
        }
        const int pos = run[d] + __popcll(eq & below);
        __builtin_amdgcn_wave_barrier();
        // the highest lane of each digit advances its run (one writer per digit)
        if (ok && (eq >> lane) == 1ull) run[d] += __popcll(eq);
        __builtin_amdgcn_wave_barrier();
        if (ok) {
            keys_out[pos] = k;
            vals_out[pos] = v;
        }
    }
}

template <typename K>
__global__ __launch_bounds__(kW) void k_copy_pairs(const K *__restrict__ k0, const int32_t *__restrict__ v0, int64_t n,
                                                   K *__restrict__ k1, int32_t *__restrict__ v1) {
    for (int64_t i = (int64_t)blockIdx.x * kW + threadIdx.x; i < n; i += (int64_t)gridDim.x * kW) {
        k1[i] = k0[i];
        v1[i] = v0[i];
    }
}

template <typename K>
size_t sort_tmp_layout(int64_t n, size_t *off_sums, size_t *off_keys, size_t *off_vals) {
    const int64_t nt = n > 0 ? tiles_of(n) : 1;
    const int64_t nh = (int64_t)kMaxBins * nt;
    size_t b = align256((size_t)nh * sizeof(int32_t));                  // histogram / offsets
    *off_sums = b;
    b += align256((size_t)(tiles_of(nh) + 1) * sizeof(int32_t));        // their tile sums
    *off_keys = b;
    b += align256((size_t)(n > 0 ? n : 1) * sizeof(K));                 // scratch keys
    *off_vals = b;
    b += align256((size_t)(n > 0 ? n : 1) * sizeof(int32_t));           // scratch values
    return b;
}

template <typename K>
hipError_t sort_impl(void *tmp, K *k0, K *k1, int32_t *v0, int32_t *v1, int64_t n, int begin_bit, int end_bit,
                     hipStream_t s) {
    if (n <= 0) return hipSuccess;
    if (n > (int64_t)INT32_MAX) return hipErrorInvalidValue;  // the digit offsets are int32
    size_t os, ok_, ov;
    (void)sort_tmp_layout<K>(n, &os, &ok_, &ov);
    char *t = static_cast<char *>(tmp);
    int32_t *hist = reinterpret_cast<int32_t *>(t);
    int32_t *sums = reinterpret_cast<int32_t *>(t + os);
    K *ks = reinterpret_cast<K *>(t + ok_);
    int32_t *vs = reinterpret_cast<int32_t *>(t + ov);
    const int bits = end_bit - begin_bit;
    const int P = bits <= 0 ? 0 : (bits + 7) / 8;
    if (P == 0) {  // nothing to sort by: the output is the input
        const int64_t g = (n + kW - 1) / kW;
        hipLaunchKernelGGL((k_copy_pairs<K>), dim3((unsigned)(g < kMaxGrid ? g : kMaxGrid)), dim3(kW), 0, s, k0, v0, n,
                           k1, v1);
        return hipGetLastError();
    }
    const int db = (bits + P - 1) / P;
    const int64_t nt = tiles_of(n);
    const K *ksrc = k0;
    const int32_t *vsrc = v0;
    for (int j = 1; j <= P; ++j) {
        const int lo = begin_bit + (j - 1) * db;
        const int w = (lo + db > end_bit) ? end_bit - lo : db;
        // the last pass lands in (k1, v1): with P odd the destinations run k1, ks, k1, ...; even ks, k1, ...
        const bool to1 = (P % 2 == 1) == (j % 2 == 1);
        K *kd = to1 ? k1 : ks;
        int32_t *vd = to1 ? v1 : vs;
        const int64_t nhw = ((int64_t)1 << w) * nt;
        hipLaunchKernelGGL((k_digit_hist<K>), dim3((unsigned)nt), dim3(kW), 0, s, ksrc, n, lo, w, hist, nt);
        hipError_t e = scan_impl<int32_t, int32_t>(hist, hist, nhw, nullptr, sums, s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL((k_digit_scatter<K>), dim3((unsigned)nt), dim3(kW), 0, s, ksrc, vsrc, n, lo, w, hist, nt, kd,
                           vd);
        ksrc = kd;
        vsrc = vd;
    }
    return hipGetLastError();
}

}  // namespace

hipError_t slot_fill(void *p, int64_t nwords, unsigned int value, hipStream_t s) {
    if (nwords <= 0) return hipSuccess;
    const int64_t g = (nwords + kW * 16 - 1) / (kW * 16);
    hipLaunchKernelGGL(k_fill, dim3((unsigned)(g < kMaxGrid ? g : kMaxGrid)), dim3(kW), 0, s,
                       static_cast<unsigned int *>(p), nwords, value);
    return hipGetLastError();
}

size_t slot_scan_temp_bytes(int64_t n) { return align256((size_t)(tiles_of(n > 0 ? n : 1) + 1) * sizeof(int64_t)); }

hipError_t slot_exclusive_scan(const int32_t *in, int64_t *out, int64_t n, int64_t *total, void *tmp, hipStream_t s) {
    return scan_impl<int32_t, int64_t>(in, out, n, total, tmp, s);
}

size_t slot_sort_temp_bytes(int64_t n, int key_bytes) {
    size_t a, b, c;
    return key_bytes == 8 ? sort_tmp_layout<unsigned long long>(n, &a, &b, &c) : sort_tmp_layout<unsigned int>(n, &a, &b, &c);
}

hipError_t slot_sort_pairs(void *tmp, const unsigned long long *k0, unsigned long long *k1, const int32_t *v0,
                           int32_t *v1, int64_t n, int begin_bit, int end_bit, hipStream_t s) {
    return sort_impl<unsigned long long>(tmp, const_cast<unsigned long long *>(k0), k1, const_cast<int32_t *>(v0), v1,
                                         n, begin_bit, end_bit, s);
}

hipError_t slot_sort_pairs(void *tmp, const unsigned int *k0, unsigned int *k1, const int32_t *v0, int32_t *v1,
                           int64_t n, int begin_bit, int end_bit, hipStream_t s) {
    return sort_impl<unsigned int>(tmp, const_cast<unsigned int *>(k0), k1, const_cast<int32_t *>(v0), v1, n,
                                   begin_bit, end_bit, s);
}

}  // namespace bre
