// bre_api.hip — C ABI of libbre.so (include/bre.h): context, device memory, build and gather
// orchestration on one HIP stream.  No exceptions cross the ABI; every failure is a status code
// plus a message for bre_last_error().
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <string>
#include <initializer_list>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/bre.h"
#include "bre_device.h"
#include "bre_trace.h"

using namespace bre;

#ifndef BRE_KERNEL_READBACK
#define BRE_KERNEL_READBACK 1
#endif

namespace {

struct DevMem {
    void *ptr = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        cap = 0;
        size_t want = bytes + bytes / 4 + 256;
        hipError_t e = hipMalloc(&ptr, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        cap = 0;
    }
    template <typename T>
    T *as() const {
        return static_cast<T *>(ptr);
    }
};

}  // namespace

struct bre_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    std::string err;
    // options
    bool counters = false;
    bool timing = false;
    int kernel = 0;
    int leaf_size = 1;
    int sqrt_mode = 0;
    int split = 256;         // work roots per packet (r2: 64 with the rotated block map, C2 +42% over 8; 256 +2% on the final kernel, partials 3 KB per segment)
    bool prefilter = true;
    int stack_cap = 0;       // internal: traversal stack entries to use (0 = all; tests force an overflow)
    int block_map = 3;       // internal: tile kernel block mapping (GatherArgs::block_map): 3 LPT (roots by size), 1 rotated
    int tscan = -1;          // internal: tile kernel transposed-scan threshold (GatherArgs::tscan), 0 = off,
                             // -1 = by the gather's MaxDistance (tscan_for; 4 fixed until round 6)
                             // (round 5: 4 over 6, C2 +0.5%, C3 +4.8%, profiles/r5/run20, run22)
    int margin = 1;          // internal: tile kernel prefilter margins (GatherArgs::margin)
    int split_records = 0;   // internal: 1 = never carry the power in BeamRec (A/B of the layouts)
    int tile_axis = 1;       // internal (option 112): per-lane tile line reject (GatherArgs::tileax), 1 = on (default since round 4), 0 = off
    int film_compose = 1;    // internal (option 114): 1 = per-pixel deterministic compose (default), 0 = float atomics (A/B)
    int occupancy = 6;       // tile kernel register budget (min waves per SIMD): 6 with the lane ray in registers (r2 final, 77 VGPRs; explore38)
    int sort_key = 4;        // segment coherence sort key (SegSort::key_mode; 4 measured best at C2)
    int shard_rank = 0, shard_count = 1;  // camera-pass image-tile shard of this context
    int shard_block = 1;                  // tiles per side of the blocks dealt to the shards
    int shard_mode = 0;                   // BRE_OPT_SHARD_MODE: 0 image tiles, 1 packet ranges
    int roots_split = -1;  // split the roots buffer was computed for (-1: stale)
    bool nodes4_ok = false;  // nodes4 holds the 4-wide view of the current tree
    int leaf2 = 64;          // kernel 0: beams per leaf tile of the tile tree (64 best at C2)
    int beam_key = 2;        // internal: tree order of the build (BuildBuffers::beam_key): 2 / 1 (start, end) Hilbert / Morton, 0 centroid
    int64_t partial_cap = (int64_t)4 << 30;  // tile kernel: bytes of per-subtree partials per launch (4 GiB)
    unsigned int *flags_host = nullptr;  // pinned copy of DevCounters::flags (check_flags)
    unsigned int *rb_host = nullptr;     // pinned words of read_small (kernel readback)
    int kernel_readback = BRE_KERNEL_READBACK;  // internal (option 118): read_small through k_readback
    int coarse_keys = 0;  // internal (option 121): 1 = the tree-order and segment sorts on the keys' top 48
                          // bits (6 radix passes instead of 8 each; round 6, profiles/r6/e13); 0 (default)
                          // all bits.  Off: its first form hung the full C5 render (the hierarchy saw
                          // unsorted low bits) and the fixed form is not yet measured on the GPU.
    int slot_passes = 1;  // internal (option 119): the pass chain's scans, sorts and fills by the one-wave
                          // primitives (bre_slot.hip, default) / 0 rocPRIM and hipMemsetAsync (A/B)
    // kernel 5: capsule-chunk index, rebuilt per gather (bre_chunk.hip)
    int chunk_len = 400;   // chunk length in units of E / 100
    int chunk_leaf = 1;    // chunks per LBVH leaf
    DevMem ch_bounds, ch_counts, ch_offsets, ch_range, ch_scan_tmp, ch_box, ch_cent, ch_slo, ch_shi, ch_par,
        ch_recs, ch_cpar, ch_nodes;
    int64_t n_chunks = 0;
    // coherence sort of the camera-pass segments before the gather (bre_sort.hip)
    bool sort_segments = true;
    DevMem ss_bounds, ss_keys, ss_keys_alt, ss_vals, ss_vals_alt, ss_tmp, ss_o, ss_p, ss_d, ss_t, ss_pix;
    DevMem sp_o, sp_p, sp_d, sp_t, sp_pix, sp_index;  // this packet shard's segments (contiguous)
    DevMem px_seg, px_keys, px_keys_alt, px_vals, px_vals_alt, px_tmp;  // deterministic per-pixel compose
    // beam set
    int64_t nbeams = 0, nvalid = 0, nnodes = 0;
    BeamSet bset;  // the built set's radius layout (BeamRec)
    int built_leaf_size = 1;
    DevMem in_start, in_end, in_radius, in_power;  // staging for host-pointer uploads
    DevMem box, cent, cbounds, nvalid_buf, keys, keys_alt, vals, vals_alt, sort_tmp, leaf_parent, visit, gbox;
    DevMem recs, pow, nodes;
    // gather staging (host-pointer API)
    DevMem g_o, g_p, g_d, g_tmax, g_pix, g_accum, g_seg_rgb, g_counts;
    DevMem chk_x, chk_aux, chk_y;  // bre_device_check staging
    DevMem counters_buf, roots, roots_sh, roots_tmp, partial, pcnt, segrec, tileax, segbox, nodes4;
    // photon pass
    DevMem ph_scene, ph_counts, ph_offsets, ph_tmp, grid_dens;
    DevMem ph_s_start, ph_s_end, ph_s_radius, ph_s_power;  // single-trace photon pass: per-photon beam slots
    int photon_single = 1;  // internal (option 116): 1 single-trace photon pass (default), 0 two traces, 2..64 forced slots
    // scene geometry on the device (upload_scene): triangles, BVHAccel nodes + primitive order, lights
    DevMem sc_tris, sc_nodes, sc_prims, sc_light_tri, sc_light_func, sc_light_cdf;
    uint64_t sc_hash = 0;  // hash of the uploaded triangles (0: none)
    std::vector<unsigned char> sc_bytes;  // the uploaded triangles' bytes: a hash match is confirmed by memcmp
    DevScene sc_head;      // geometry fields of the uploaded scene
    DevScene ph_scene_host;                 // the record last copied to ph_scene
    std::vector<unsigned char> grid_bytes;  // the density grid last copied to grid_dens
    // camera pass
    DevMem cam_dev, cam_perms, cs_o, cs_p, cs_d, cs_t, cs_pix, cs_valid, cam_offs, cam_tmp, cam_flags;
    DevMem seg_o, seg_p, seg_d, seg_t, seg_pix, seg_depth;
    int64_t cam_nseg = 0;
    int64_t cam_npix = 0;
    int cam_w = -1, cam_h = -1;  // film the Halton / camera tables were prepared for
    bre_scene cam_scene;         // scene the camera tables were prepared for
    bool beams_kept = false;  // in_* hold the current beam set (bre_get_beams)
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    bre_stats stats;
    // film classes (BRE_OPT_FILM_CLASSES): 1, or BRE_FILM_CLASSES planes per film; px_cls the class per segment
    int film_classes = 1;
    DevMem px_cls;
    // the passes' own high-priority stream (option 117, PassStream below)
    int pass_priority = 1;
    hipStream_t pstream = nullptr;
    hipEvent_t fork_ev = nullptr, join_ev = nullptr;
    // bre_set_gather_after: this context's tile kernels wait for `after`'s last one (after->tile_ev)
    bre_ctx *after = nullptr;
    std::vector<bre_ctx *> followers;  // contexts whose `after` is this one (unlinked in bre_destroy)
    hipEvent_t tile_ev = nullptr;  // recorded after each tile-kernel launch (created on first use)
    bool tile_ev_valid = false;
    hipEvent_t user_ev[2] = {nullptr, nullptr};  // bre_set_gather_events
};

namespace {

bre_status fail(bre_ctx *c, bre_status st, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (c) c->err = buf;
    return st;
}

#define HIPCHK(ctx, call)                                                                                    \
    do {                                                                                                     \
        hipError_t e_ = (call);                                                                              \
        if (e_ != hipSuccess)                                                                                \
            return fail((ctx), e_ == hipErrorOutOfMemory ? BRE_ERR_OOM : BRE_ERR_HIP, "%s: %s (%s:%d)", #call, \
                        hipGetErrorString(e_), __FILE__, __LINE__);                                          \
    } while (0)

bre_status set_device(bre_ctx *c) {
    HIPCHK(c, hipSetDevice(c->device));
    return BRE_OK;
}

// Zero `bytes` (a multiple of 4) of device memory on the context's stream: a one-wave fill kernel
// (bre_slot.hip) instead of hipMemsetAsync's runtime kernel, which waits for CUs behind a concurrent
// gather (the pipelined pass chain); option 119 = 0 keeps hipMemsetAsync.
hipError_t fill_words(bre_ctx *c, void *p, size_t bytes) {
    if (!c->slot_passes || bytes % 4) return hipMemsetAsync(p, 0, bytes, c->stream);
    return slot_fill(p, (int64_t)(bytes / 4), 0u, c->stream);
}

// Small device-to-host reads of the pass chain (the photon total, the build's valid count, the camera
// pass's segment total, the sticky error flags), synchronising the context's stream.  With option 118
// a one-wave kernel stores the words into pinned host memory; otherwise hipMemcpyAsync, whose copy
// kernel (the runtime's own, with multi-wave workgroups) waited up to 32 ms for CUs behind a
// concurrent gather's one-wave blocks in the round-5 pipelined trace.
struct ReadSpans {
    const unsigned int *src[4];
    int words[4];
    int n;
};
__global__ __launch_bounds__(64) void k_readback(ReadSpans r, unsigned int *__restrict__ dst) {
    int o = 0;
    for (int i = 0; i < r.n; ++i) {
        if ((int)threadIdx.x < r.words[i]) dst[o + threadIdx.x] = r.src[i][threadIdx.x];
        o += r.words[i];
    }
}
struct HostSpan {
    void *host;
    const void *dev;
    size_t bytes;  // a multiple of 4, <= 64 words over all spans
};
bre_status read_small(bre_ctx *c, std::initializer_list<HostSpan> spans) {
    if (!c->kernel_readback) {
        for (const HostSpan &h : spans)
            HIPCHK(c, hipMemcpyAsync(h.host, h.dev, h.bytes, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        return BRE_OK;
    }
    if (!c->rb_host) {
        void *h = nullptr;
        HIPCHK(c, hipHostMalloc(&h, 64 * sizeof(unsigned int), hipHostMallocDefault));
        c->rb_host = static_cast<unsigned int *>(h);
    }
    ReadSpans r{};
    int tot = 0;
    for (const HostSpan &h : spans) {
        if (r.n == 4 || h.bytes % 4 || tot + (int)(h.bytes / 4) > 64) return fail(c, BRE_ERR_STATE, "read_small: bad span");
        r.src[r.n] = static_cast<const unsigned int *>(h.dev);
        r.words[r.n] = (int)(h.bytes / 4);
        tot += r.words[r.n++];
    }
    hipLaunchKernelGGL(k_readback, dim3(1), dim3(64), 0, c->stream, r, c->rb_host);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipStreamSynchronize(c->stream));
    int o = 0;
    for (const HostSpan &h : spans) {
        memcpy(h.host, c->rb_host + o, h.bytes);
        o += (int)(h.bytes / 4);
    }
    return BRE_OK;
}

// The photon pass (with its BVH build) and the camera pass run on a stream of the device's highest
// priority, forked from the caller's stream and joined back to it (option 117, default on): stream
// order towards the caller is unchanged, but when two contexts pipeline the render (iteration k+1's
// passes beside iteration k's gather, bench.py --pipeline 1) the dispatcher hands the passes' few
// workgroups the CUs as the gather's one-wave blocks retire, instead of queueing them behind millions
// of gather blocks (round 4: k_photons averaged 80 ms in the pipelined trace against 1.4 ms alone).
struct PassStream {
    bre_ctx *c;
    hipStream_t user = nullptr;
    PassStream(bre_ctx *c_) : c(c_) {
        if (!c->pass_priority) return;
        if (!c->pstream) {
            int least = 0, greatest = 0;
            if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) return;
            if (hipStreamCreateWithPriority(&c->pstream, hipStreamNonBlocking, greatest) != hipSuccess) {
                c->pstream = nullptr;
                return;
            }
            if (hipEventCreateWithFlags(&c->fork_ev, hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&c->join_ev, hipEventDisableTiming) != hipSuccess)
                return;
        }
        if (!c->fork_ev || !c->join_ev) return;
        if (hipEventRecord(c->fork_ev, c->stream) != hipSuccess ||
            hipStreamWaitEvent(c->pstream, c->fork_ev, 0) != hipSuccess)
            return;
        user = c->stream;
        c->stream = c->pstream;
    }
    ~PassStream() {
        if (!user) return;
        // the caller's stream waits for everything the pass queued (also on an early error return)
        (void)hipEventRecord(c->join_ev, c->pstream);
        (void)hipStreamWaitEvent(user, c->join_ev, 0);
        c->stream = user;
    }
};

// Build the BVH from device arrays (start/end/radius/power) of n beams.
bre_status build(bre_ctx *c, int64_t n, const float *start, const float *end, const float *radius,
                 const float *power) {
    c->nbeams = n;
    c->nvalid = 0;
    c->bset = BeamSet{};
    c->nnodes = 0;
    c->roots_split = -1;
    c->nodes4_ok = false;
    c->stats = bre_stats{};
    c->stats.n_beams = n;
    if (n == 0) return BRE_OK;
    if (n > (int64_t)INT32_MAX / 2)
        return fail(c, BRE_ERR_INVALID_ARG, "bre_set_beams: %lld beams exceeds the 2^30 limit of this build",
                    (long long)n);
    const size_t N = (size_t)n;
    HIPCHK(c, c->box.ensure(N * 6 * sizeof(float)));
    HIPCHK(c, c->cent.ensure(N * 3 * sizeof(float)));
    HIPCHK(c, c->cbounds.ensure(12 * sizeof(unsigned int)));
    HIPCHK(c, c->nvalid_buf.ensure(3 * sizeof(unsigned int)));
    HIPCHK(c, c->keys.ensure(N * sizeof(unsigned long long)));
    HIPCHK(c, c->keys_alt.ensure(N * sizeof(unsigned long long)));
    HIPCHK(c, c->vals.ensure(N * sizeof(int32_t)));
    HIPCHK(c, c->vals_alt.ensure(N * sizeof(int32_t)));
    const size_t tmp = sort_temp_bytes(n);
    HIPCHK(c, c->sort_tmp.ensure(tmp));
    BuildBuffers b;
    b.start = start;
    b.end = end;
    b.radius = radius;
    b.power = power;
    b.n = n;
    b.sqrt_mode = c->sqrt_mode;
    b.slot = c->slot_passes;
    b.leaf_size = c->leaf_size;
    b.beam_key = c->beam_key;
    b.box = c->box.as<float>();
    b.cent = c->cent.as<float>();
    b.cbounds = c->cbounds.as<unsigned int>();
    b.nvalid = c->nvalid_buf.as<unsigned int>();
    b.keys = c->keys.as<unsigned long long>();
    b.keys_alt = c->keys_alt.as<unsigned long long>();
    b.vals = c->vals.as<int32_t>();
    b.vals_alt = c->vals_alt.as<int32_t>();
    b.sort_tmp = c->sort_tmp.ptr;
    b.sort_tmp_bytes = c->sort_tmp.cap;
    if (c->timing) HIPCHK(c, hipEventRecord(c->ev[0], c->stream));
    HIPCHK(c, launch_prep(b, c->stream));
    // tree keys 1 / 2 (the tile kernel's tree): the first sort only groups equal centroids (a hash key,
    // bre_build.hip k_cent_hash); otherwise the centroid Morton order is the tree order
    const bool se_tree = c->kernel == 0 && c->beam_key >= 1;
    if (se_tree) {
        HIPCHK(c, launch_cent_hash(b, c->stream));
        HIPCHK(c, launch_sort(b, c->stream, 32));
    } else {
        HIPCHK(c, launch_morton(b, c->stream));
        HIPCHK(c, launch_sort(b, c->stream));
    }
    unsigned int nv[3] = {0u, 0u, 0u};  // valid beams, min / max of their radius bits (k_prep)
    {
        const bre_status rs = read_small(c, {{nv, b.nvalid, sizeof(nv)}});
        if (rs != BRE_OK) return rs;
    }
    const int64_t nvalid = nv[0];
    c->nvalid = nvalid;
    // one radius for every valid beam: the records carry the power instead (BeamRec, BeamSet)
    c->bset.uniform = (nvalid > 0 && nv[1] == nv[2] && !c->split_records) ? 1 : 0;
    std::memcpy(&c->bset.radius, &nv[1], sizeof(float));
    if (!c->bset.uniform) c->bset.radius = 0.f;
    b.uniform_radius = c->bset.uniform;
    c->stats.n_beams_valid = nvalid;
    if (nvalid == 0) return BRE_OK;
    if (se_tree) {
        // tree order by (start, end): group boxes from the centroid order, then the second sort
        HIPCHK(c, c->gbox.ensure(N * 6 * sizeof(float)));
        b.gbox = c->gbox.as<float>();
        HIPCHK(c, launch_tree_key(b, nvalid, c->stream));
        b.key_lo = c->coarse_keys ? 16 : 0;  // the hierarchy compares the bits the sort ordered
        HIPCHK(c, launch_sort(b, c->stream, 64, b.key_lo));
    } else {
        b.beam_key = 0;
    }
    // kernel 0 runs the tile kernel on one tree of leaf2-beam tiles; kernels 2 / 4 / 5 on a tree of
    // BRE_OPT_LEAF_SIZE-beam leaves
    const int K = c->kernel == 0 ? c->leaf2 : c->leaf_size;
    b.leaf_size = K;  // the hierarchy kernels size their work by it: must match the buffers below
    const int64_t nleaf = (nvalid + K - 1) / K;
    const int64_t nnodes = nleaf > 1 ? nleaf - 1 : 1;
    HIPCHK(c, c->recs.ensure((size_t)nvalid * sizeof(BeamRec)));
    HIPCHK(c, c->pow.ensure((size_t)nvalid * sizeof(float4)));
    HIPCHK(c, c->nodes.ensure((size_t)nnodes * sizeof(Node)));
    HIPCHK(c, c->leaf_parent.ensure((size_t)nleaf * sizeof(int32_t)));
    HIPCHK(c, c->visit.ensure((size_t)nnodes * sizeof(unsigned int)));
    b.recs = c->recs.as<BeamRec>();
    b.pow = c->pow.as<float4>();
    b.nodes = c->nodes.as<Node>();
    b.leaf_parent = c->leaf_parent.as<int32_t>();
    b.visit = c->visit.as<unsigned int>();
    b.nodes_cap = c->nodes.cap / sizeof(Node);
    b.leaf_parent_cap = c->leaf_parent.cap / sizeof(int32_t);
    b.visit_cap = c->visit.cap / sizeof(unsigned int);
    HIPCHK(c, launch_pack(b, nvalid, c->stream));
    HIPCHK(c, launch_hierarchy(b, nvalid, c->stream));
    if (c->timing) {
        HIPCHK(c, hipEventRecord(c->ev[1], c->stream));
        HIPCHK(c, hipEventSynchronize(c->ev[1]));
        float ms = 0.f;
        HIPCHK(c, hipEventElapsedTime(&ms, c->ev[0], c->ev[1]));
        c->stats.build_ms = ms;
    }
    c->nnodes = nnodes;
    c->built_leaf_size = K;
    c->stats.n_nodes = nnodes;
    if (c->kernel == 0 || c->kernel == 4) {
        // the tile kernel's work roots and 4-wide view, here on the build's stream: with two contexts
        // pipelined they overlap the other context's gather instead of preceding this one's
        HIPCHK(c, c->roots.ensure(sizeof(int32_t) * (kMaxSplit + 1)));
        HIPCHK(c, c->roots_tmp.ensure(roots_scratch_bytes()));
        HIPCHK(c, launch_roots(c->nodes.as<Node>(), c->split, c->roots.as<int32_t>(), c->roots_tmp.ptr, c->stream));
        c->roots_split = c->split;
        HIPCHK(c, c->nodes4.ensure(sizeof(Node4) * (size_t)nnodes));
        HIPCHK(c, launch_collapse4(c->nodes.as<Node>(), nnodes, c->nodes4.as<Node4>(), c->stream));
        c->nodes4_ok = true;
    }
    return BRE_OK;
}

bre_status read_counters(bre_ctx *c, DevCounters *ctr);
bre_status check_flags(bre_ctx *c);

// Kernel 5: build the capsule-chunk index for this gather's segments and R, then gather through it
// (bre_chunk.hip).  Every array is a context buffer reused across calls; the beam build's sort
// scratch (keys / vals / sort_tmp / leaf_parent / visit) is reused, it is dead after the build.
bre_status gather_chunk(bre_ctx *c, const GatherArgs &a) {
    const int64_t np = c->nvalid;
    if (c->timing) HIPCHK(c, hipEventRecord(c->ev[2], c->stream));
    ChunkBuild cb;
    HIPCHK(c, c->ch_bounds.ensure(12 * sizeof(unsigned int)));
    HIPCHK(c, c->ch_counts.ensure((size_t)(np + 1) * sizeof(int32_t)));
    HIPCHK(c, c->ch_offsets.ensure((size_t)(np + 1) * sizeof(int64_t)));
    HIPCHK(c, c->ch_range.ensure((size_t)(2 * np + 2) * sizeof(float)));
    const size_t st = chunk_scan_temp_bytes(np);
    HIPCHK(c, c->ch_scan_tmp.ensure(st + 16));
    cb.parents = c->recs.as<BeamRec>();
    cb.bset = c->bset;
    cb.nparents = np;
    cb.seg_o = a.o;
    cb.seg_p = a.p;
    cb.nseg = a.nseg;
    cb.R = a.R;
    cb.len_factor = (float)c->chunk_len / 100.f;
    cb.seg_bounds = c->ch_bounds.as<unsigned int>();
    cb.cbounds = c->ch_bounds.as<unsigned int>() + 6;
    cb.counts = c->ch_counts.as<int32_t>();
    cb.offsets = c->ch_offsets.as<int64_t>();
    cb.range = c->ch_range.as<float>();
    cb.scan_tmp = c->ch_scan_tmp.ptr;
    cb.scan_tmp_bytes = st;
    HIPCHK(c, launch_chunk_count(cb, c->stream));
    int64_t total = 0;
    HIPCHK(c, hipMemcpyAsync(&total, cb.offsets + np, sizeof(total), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (total > ((int64_t)1 << 30))
        return fail(c, BRE_ERR_INVALID_ARG, "bre_gather: kernel 5 needs %lld chunks (> 2^30); raise BRE_OPT_CHUNK_LEN "
                    "or use kernel 0", (long long)total);
    c->n_chunks = total;
    if (total == 0) {
        HIPCHK(c, launch_zero_outputs(a, c->stream));
        return BRE_OK;
    }
    const size_t C = (size_t)total;
    const int K = c->chunk_leaf;
    const int64_t nleaf = (total + K - 1) / K;
    const int64_t nnodes = nleaf > 1 ? nleaf - 1 : 1;
    HIPCHK(c, c->ch_box.ensure(C * 6 * sizeof(float)));
    HIPCHK(c, c->ch_cent.ensure(C * 3 * sizeof(float)));
    HIPCHK(c, c->ch_slo.ensure(C * sizeof(float)));
    HIPCHK(c, c->ch_shi.ensure(C * sizeof(float)));
    HIPCHK(c, c->ch_par.ensure(C * sizeof(int32_t)));
    HIPCHK(c, c->keys.ensure(C * sizeof(unsigned long long)));
    HIPCHK(c, c->keys_alt.ensure(C * sizeof(unsigned long long)));
    HIPCHK(c, c->vals.ensure(C * sizeof(int32_t)));
    HIPCHK(c, c->vals_alt.ensure(C * sizeof(int32_t)));
    const size_t sb = sort_temp_bytes(total);
    HIPCHK(c, c->sort_tmp.ensure(sb + 16));
    HIPCHK(c, c->ch_recs.ensure(C * sizeof(ChunkRec)));
    HIPCHK(c, c->ch_cpar.ensure(C * sizeof(int32_t)));
    HIPCHK(c, c->ch_nodes.ensure((size_t)nnodes * sizeof(Node)));
    HIPCHK(c, c->leaf_parent.ensure((size_t)nleaf * sizeof(int32_t)));
    HIPCHK(c, c->visit.ensure((size_t)nnodes * sizeof(unsigned int)));
    HIPCHK(c, launch_chunk_emit(cb, c->ch_box.as<float>(), c->ch_cent.as<float>(), c->ch_slo.as<float>(),
                                c->ch_shi.as<float>(), c->ch_par.as<int32_t>(), c->stream));
    BuildBuffers bb{};
    bb.n = total;
    bb.leaf_size = K;
    bb.box = c->ch_box.as<float>();
    bb.cent = c->ch_cent.as<float>();
    bb.cbounds = cb.cbounds;
    bb.keys = c->keys.as<unsigned long long>();
    bb.keys_alt = c->keys_alt.as<unsigned long long>();
    bb.vals = c->vals.as<int32_t>();
    bb.vals_alt = c->vals_alt.as<int32_t>();
    bb.sort_tmp = c->sort_tmp.ptr;
    bb.sort_tmp_bytes = sb;
    bb.leaf_parent = c->leaf_parent.as<int32_t>();
    bb.visit = c->visit.as<unsigned int>();
    bb.recs = reinterpret_cast<BeamRec *>(c->ch_recs.as<ChunkRec>());  // same leading lo / hi layout
    bb.nodes = c->ch_nodes.as<Node>();
    bb.nodes_cap = c->ch_nodes.cap / sizeof(Node);
    bb.leaf_parent_cap = c->leaf_parent.cap / sizeof(int32_t);
    bb.visit_cap = c->visit.cap / sizeof(unsigned int);
    HIPCHK(c, launch_morton(bb, c->stream));
    HIPCHK(c, launch_sort(bb, c->stream));
    HIPCHK(c, launch_chunk_pack(cb, total, bb.vals_alt, bb.box, c->ch_slo.as<float>(), c->ch_shi.as<float>(),
                                c->ch_par.as<int32_t>(), c->ch_recs.as<ChunkRec>(), c->ch_cpar.as<int32_t>(),
                                c->stream));
    HIPCHK(c, launch_hierarchy(bb, total, c->stream));
    ChunkGatherArgs g;
    g.nseg = a.nseg;
    g.o = a.o;
    g.p = a.p;
    g.d = a.d;
    g.tmax = a.tmax;
    g.pixel = a.pixel;
    g.R = a.R;
    g.npix = a.npix;
    g.accum = a.accum;
    g.seg_rgb = a.seg_rgb;
    g.seg_counts = a.seg_counts;
    g.chunks = c->ch_recs.as<ChunkRec>();
    g.chunk_parent = c->ch_cpar.as<int32_t>();
    g.parents = c->recs.as<BeamRec>();
    g.pow = c->pow.as<float4>();
    g.nodes = c->ch_nodes.as<Node>();
    g.nchunks = total;
    g.leaf_size = K;
    g.prefilter = c->prefilter;
    g.ctr = a.ctr;
    HIPCHK(c, launch_gather_chunk(g, c->counters, c->stream));
    if (c->timing) HIPCHK(c, hipEventRecord(c->ev[3], c->stream));
    return read_counters(c, a.ctr);
}

// The counter block of the context: zeroed once at allocation; per gather only the counters are
// zeroed, the sticky `flags` word stays until check_flags has read it.
bre_status counters_block(bre_ctx *c, DevCounters **out) {
    if (!c->counters_buf.ptr) {
        HIPCHK(c, c->counters_buf.ensure(sizeof(DevCounters)));
        HIPCHK(c, fill_words(c, c->counters_buf.ptr, sizeof(DevCounters)));
    }
    *out = c->counters_buf.as<DevCounters>();
    static_assert(offsetof(DevCounters, flags) % 4 == 0, "DevCounters: word-aligned flags");
    HIPCHK(c, fill_words(c, *out, offsetof(DevCounters, flags)));
    return BRE_OK;
}

// Synchronise the stream and turn the device's sticky error flags into a status (then clear them).
// Every synchronising entry point ends here, so a traversal-stack overflow or a bad pixel index of
// an earlier asynchronous gather is reported whatever the counters option (never silent).
bre_status check_flags(bre_ctx *c) {
    if (!c->counters_buf.ptr) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        return BRE_OK;
    }
    if (!c->flags_host) {
        void *h = nullptr;
        HIPCHK(c, hipHostMalloc(&h, sizeof(unsigned int), hipHostMallocDefault));
        c->flags_host = static_cast<unsigned int *>(h);
    }
    unsigned int *dflags = &c->counters_buf.as<DevCounters>()->flags;
    {
        const bre_status rs = read_small(c, {{c->flags_host, dflags, sizeof(unsigned int)}});
        if (rs != BRE_OK) return rs;
    }
    const unsigned int f = *c->flags_host;
    if (f == 0) return BRE_OK;
    HIPCHK(c, fill_words(c, dflags, sizeof(unsigned int)));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (f & kFlagStack)
        return fail(c, BRE_ERR_STATE, "bre_gather: traversal stack overflow (BVH deeper than the stack): contributions "
                    "were dropped");
    return fail(c, BRE_ERR_INVALID_ARG, "bre_gather: seg_pixel out of [0, npix): segments were skipped");
}

// The transposed-scan threshold by the gather's MaxDistance (option 108 = -1, the default since round 6).
// A tile is scanned transposed when its on-lanes * 8 < kept beams * t; the best t falls as the pass rate of
// the lane tests rises, and that rate grows with MaxDistance against the packets' bundle spread (~0.06-0.12
// in the unit-box scenes).  Measured on one box (profiles/r6/e6, sums bit-identical for every t): C2
// iteration 0 (MaxDistance 0.02) 252.8 / 254.2 / 257.3 ms for t = 3 / 4 / 5, iteration 15 (0.005) 110.4 /
// 108.9 / 108.3 ms; C3 iteration 0 (0.02) 2965 / 3001 / 3064 ms.
int tscan_for(float maxd) { return maxd >= 0.015f ? 3 : (maxd >= 0.008f ? 4 : 5); }

bre_status gather_device(bre_ctx *c, int64_t nseg, const float *o, const float *p, const float *d, const float *tmax,
                         const int32_t *pixel, float R, int64_t npix, float *accum, float *seg_rgb,
                         int32_t *seg_counts, const int32_t *seg_index = nullptr) {
    if (nseg < 0 || npix < 0) return fail(c, BRE_ERR_INVALID_ARG, "bre_gather: negative size");
    if (nseg > 0 && (!o || !p || !d || !tmax))
        return fail(c, BRE_ERR_INVALID_ARG, "bre_gather: null segment array");
    if (accum && !pixel) return fail(c, BRE_ERR_INVALID_ARG, "bre_gather: accum_rgb given without seg_pixel");
    DevCounters *ctr = nullptr;
    bre_status st = counters_block(c, &ctr);
    if (st != BRE_OK) return st;
    GatherArgs a{};
    a.nseg = nseg;
    a.o = o;
    a.p = p;
    a.d = d;
    a.tmax = tmax;
    a.pixel = pixel;
    a.R = R;
    a.npix = npix;
    a.accum = accum;
    a.seg_rgb = seg_rgb;
    a.seg_counts = seg_counts;
    a.seg_index = seg_index;
    a.recs = c->recs.as<BeamRec>();
    a.pow = c->pow.as<float4>();
    a.bset = c->bset;
    a.nodes = c->nodes.as<Node>();
    a.nvalid = c->nvalid;
    a.leaf_size = c->built_leaf_size;
    a.ctr = ctr;
    a.split = c->split;
    a.prefilter = c->prefilter;
    a.occupancy = c->occupancy;
    a.block_map = c->block_map;
    a.tscan = c->tscan >= 0 ? c->tscan : tscan_for(R + c->bset.radius);
    a.margin = c->margin;
    a.stack_cap = c->stack_cap;
    c->stats.n_segments = nseg;
    if (c->nvalid == 0) {
        // empty PhotonBeamBVH: Intersect returns nothing (photonbeambvh.cpp:687)
        HIPCHK(c, launch_zero_outputs(a, c->stream));
        return BRE_OK;
    }
    int kernel = c->kernel;
    // work-root shards split the tile kernel's work roots: kernels 2 and 5 have none, and would gather
    // every segment against every beam on every shard (films summing to count x the image)
    if (c->shard_mode == 2 && c->shard_count > 1 && (kernel == 2 || kernel == 5))
        return fail(c, BRE_ERR_STATE, "work-root shards (BRE_OPT_SHARD_MODE 2) need the tile kernel (BRE_OPT_KERNEL 0 or 4)");
    if (kernel == 5) {
        if (seg_index) return fail(c, BRE_ERR_STATE, "kernel 5 gathers in the caller's order only");
        return gather_chunk(c, a);
    }
    if (kernel == 0) kernel = 4;  // the tile kernel on the tile tree built for kernel 0
    if (kernel == 2 && seg_index) return fail(c, BRE_ERR_STATE, "kernel 2 gathers in the caller's order only");
    if (kernel == 2) {
        if (c->timing) HIPCHK(c, hipEventRecord(c->ev[2], c->stream));
        HIPCHK(c, launch_gather(a, kernel, c->counters, c->stream));
        if (c->timing) HIPCHK(c, hipEventRecord(c->ev[3], c->stream));
        return read_counters(c, a.ctr);
    }
    // The tile kernel keeps S partial sums per segment (12 B each, + 8 B of counts when asked for).
    // A gather of many segments runs as consecutive launches over whole-packet ranges, so that the
    // partials stay within partial_cap (4 GiB: C2's ~0.6M segments in one launch, C4's ~9.6M in 7)
    // and the grid within HIP's 2^32 work items.  Every segment's sum is still its subtrees'
    // partials added in root order by k_reduce: the per-segment results do not depend on the split.
    const bool want_cnt = c->counters || seg_counts;
    // work-root shards (BRE_OPT_SHARD_MODE 2): this shard takes every count-th work root of the
    // size-ordered list (rank, rank + count, ...) for ALL segments, so its waves sweep whole subtrees
    // with every packet, as one GPU does; the per-segment sums are this shard's subtrees' share
    const bool rshard = c->shard_mode == 2 && c->shard_count > 1;
    const int S_eff = rshard ? (c->split + c->shard_count - 1) / c->shard_count : c->split;
    const size_t per_seg = (size_t)S_eff * (12 + (want_cnt ? 8 : 0));
    int64_t chunk = c->partial_cap / (int64_t)per_seg / 64 * 64;
    // the exact stage addresses a launch's SegRec records with 32-bit byte offsets (BRE_BUF_LOADS):
    // at most 2^26 segments (64 B each) per launch
    if (chunk > ((int64_t)1 << 26)) chunk = (int64_t)1 << 26;
    if (chunk < 64) chunk = 64;
    if (chunk > nseg) chunk = nseg;
    HIPCHK(c, c->roots.ensure(sizeof(int32_t) * (kMaxSplit + 1)));
    HIPCHK(c, c->partial.ensure(sizeof(float) * 3 * (size_t)chunk * (size_t)S_eff));
    if (c->roots_split != c->split) {
        HIPCHK(c, c->roots_tmp.ensure(roots_scratch_bytes()));
        HIPCHK(c, launch_roots(c->nodes.as<Node>(), c->split, c->roots.as<int32_t>(), c->roots_tmp.ptr, c->stream));
        c->roots_split = c->split;
    }
    if (!c->nodes4_ok) {
        // the tile kernel's 4-wide view of the tree (Node4), once per build
        HIPCHK(c, c->nodes4.ensure(sizeof(Node4) * (size_t)c->nnodes));
        HIPCHK(c, launch_collapse4(c->nodes.as<Node>(), c->nnodes, c->nodes4.as<Node4>(), c->stream));
        c->nodes4_ok = true;
    }
    a.nodes4 = c->nodes4.as<Node4>();
    a.roots = c->roots.as<int32_t>();
    if (rshard) {
        HIPCHK(c, c->roots_sh.ensure(sizeof(int32_t) * (kMaxSplit + 1)));
        HIPCHK(c, launch_roots_shard(c->roots.as<int32_t>(), c->split, c->shard_rank, c->shard_count, S_eff,
                                     c->roots_sh.as<int32_t>(), c->stream));
        a.roots = c->roots_sh.as<int32_t>();
        a.split = S_eff;
    }
    a.partial = c->partial.as<float>();
    HIPCHK(c, c->segrec.ensure(sizeof(SegRec) * (size_t)((chunk + 63) / 64 * 64)));  // whole packets
    a.segrec = c->segrec.as<SegRec>();
    if (want_cnt) {
        HIPCHK(c, c->pcnt.ensure(sizeof(int32_t) * 2 * (size_t)chunk * (size_t)S_eff));
        a.pcnt = c->pcnt.as<int32_t>();
    }
    if (c->tile_axis && a.leaf_size > 0) {
        const int64_t ntiles = (c->nvalid + a.leaf_size - 1) / a.leaf_size;
        HIPCHK(c, c->tileax.ensure(sizeof(TileAxis) * (size_t)ntiles));
        HIPCHK(c, c->segbox.ensure(sizeof(unsigned int) * 8));
        a.tileax = c->tileax.as<TileAxis>();
        a.segbox = c->segbox.as<unsigned int>();
    }
    if (c->timing) HIPCHK(c, hipEventRecord(c->ev[2], c->stream));
    if (!c->tile_ev) HIPCHK(c, hipEventCreateWithFlags(&c->tile_ev, hipEventDisableTiming));
    for (int64_t off = 0; off < nseg; off += chunk) {
        GatherArgs ac = a;
        // pipelined contexts (bre_set_gather_after): the first launch waits for the other context's last
        // tile kernel, the last one marks this context's
        ac.wait_ev = (off == 0 && c->after && c->after->tile_ev_valid) ? c->after->tile_ev : nullptr;
        ac.done_ev = off + chunk >= nseg ? c->tile_ev : nullptr;
        ac.user_start = off == 0 ? c->user_ev[0] : nullptr;
        ac.user_end = off + chunk >= nseg ? c->user_ev[1] : nullptr;
        ac.nseg = std::min(chunk, nseg - off);
        ac.o = o + 3 * off;
        ac.p = p + 3 * off;
        ac.d = d + 3 * off;
        ac.tmax = tmax + off;
        ac.pixel = pixel ? pixel + off : nullptr;
        if (seg_index) {
            ac.seg_index = seg_index + off;  // outputs are addressed through the index
        } else {
            ac.seg_rgb = seg_rgb ? seg_rgb + 3 * off : nullptr;
            ac.seg_counts = seg_counts ? seg_counts + 2 * off : nullptr;
        }
        HIPCHK(c, launch_gather(ac, kernel, c->counters, c->stream));
    }
    c->tile_ev_valid = true;
    if (c->timing) HIPCHK(c, hipEventRecord(c->ev[3], c->stream));
    return read_counters(c, a.ctr);
}

// With counters or timing on, copy the counter block back (synchronising) into the stats.
bre_status read_counters(bre_ctx *c, DevCounters *ctr) {
    if (!(c->timing || c->counters)) return BRE_OK;
    DevCounters h;
    HIPCHK(c, hipMemcpyAsync(&h, ctr, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->timing) {
        float ms = 0.f;
        HIPCHK(c, hipEventElapsedTime(&ms, c->ev[2], c->ev[3]));
        c->stats.gather_ms = ms;
    }
    c->stats.candidates = (int64_t)h.candidates;
    c->stats.contributions = (int64_t)h.contributions;
    c->stats.node_visits = (int64_t)h.node_visits;
    c->stats.leaf_visits = (int64_t)h.leaf_visits;
    c->stats.beam_evals = (int64_t)h.beam_evals;
    c->stats.ccp_wave_evals = (int64_t)h.ccp_wave_evals;
    c->stats.prefilter_rejects = (int64_t)h.prefilter_rejects;
    c->stats.useful_beam_evals = (int64_t)h.useful_beam_evals;
    c->stats.max_stack_depth = (int64_t)h.max_stack;
    c->stats.redo_items = 0;
    c->stats.queued_pairs = (int64_t)h.queued_pairs;
    c->stats.n_chunks = c->n_chunks;
    return check_flags(c);
}

// exclusive scan of the camera slots' valid flags into cam_offs
hipError_t rocprim_free_total_scan(bre_ctx *c, const CamSlots &cs, int64_t nslots, int max_depth) {
    return launch_camera_scan(c->cam_tmp.ptr, c->cam_tmp.cap, cs, nslots, max_depth, c->cam_offs.as<int64_t>(),
                              c->stream, c->slot_passes != 0);
}

}  // namespace

// bre_set_gather_after links: guarded, since the two contexts may be driven from two host threads
static std::mutex &link_mu() {
    static std::mutex m;
    return m;
}
static void unlink_follower(bre_ctx *lead, bre_ctx *f) {
    auto &v = lead->followers;
    v.erase(std::remove(v.begin(), v.end(), f), v.end());
}

extern "C" {

int bre_abi_version(void) { return BRE_ABI_VERSION; }

bre_status bre_create(int device, bre_ctx **out) {
    if (!out) return BRE_ERR_INVALID_ARG;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return BRE_ERR_NO_DEVICE;
    if (device < 0 || device >= count) return BRE_ERR_NO_DEVICE;
    bre_ctx *c = new bre_ctx();
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return BRE_ERR_HIP;
    }
    c->own_stream = true;
    for (auto &e : c->ev) {
        if (hipEventCreate(&e) != hipSuccess) {
            delete c;
            return BRE_ERR_HIP;
        }
    }
    *out = c;
    return BRE_OK;
}

void bre_destroy(bre_ctx *c) {
    if (!c) return;
    {
        // a pipelined partner must not keep waiting on this context's event once it is gone
        std::lock_guard<std::mutex> lk(link_mu());
        for (bre_ctx *f : c->followers) f->after = nullptr;
        if (c->after) unlink_follower(c->after, c);
    }
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    DevMem *all[] = {&c->in_start, &c->in_end, &c->in_radius, &c->in_power, &c->box,      &c->cent,
                     &c->cbounds,  &c->nvalid_buf, &c->keys,  &c->keys_alt, &c->vals,     &c->vals_alt,
                     &c->sort_tmp, &c->leaf_parent, &c->visit, &c->recs,    &c->pow,      &c->nodes,
                     &c->g_o,      &c->g_p,    &c->g_d,       &c->g_tmax,   &c->g_pix,    &c->g_accum,
                     &c->g_seg_rgb, &c->g_counts, &c->counters_buf, &c->roots, &c->partial, &c->pcnt, &c->segrec,
                     &c->tileax, &c->segbox, &c->nodes4, &c->roots_sh, &c->roots_tmp,
                     &c->ph_scene, &c->ph_counts, &c->ph_offsets, &c->ph_tmp, &c->ph_s_start, &c->ph_s_end, &c->ph_s_radius, &c->ph_s_power, &c->grid_dens, &c->cam_dev, &c->cam_perms,
                     &c->cs_o, &c->cs_p, &c->cs_d, &c->cs_t, &c->cs_pix, &c->cs_valid, &c->cam_offs,
                     &c->cam_tmp, &c->cam_flags, &c->seg_o, &c->seg_p, &c->seg_d, &c->seg_t, &c->seg_pix,
                     &c->seg_depth, &c->ch_bounds, &c->ch_counts,
                     &c->ch_offsets, &c->ch_range, &c->ch_scan_tmp, &c->ch_box, &c->ch_cent, &c->ch_slo, &c->ch_shi,
                     &c->ch_par, &c->ch_recs, &c->ch_cpar, &c->ch_nodes, &c->ss_bounds, &c->ss_keys,
                     &c->ss_keys_alt, &c->ss_vals, &c->ss_vals_alt, &c->ss_tmp, &c->ss_o, &c->ss_p, &c->ss_d,
                     &c->ss_t, &c->ss_pix, &c->sp_o, &c->sp_p, &c->sp_d, &c->sp_t, &c->sp_pix, &c->sp_index,
                     &c->gbox, &c->sc_tris, &c->sc_nodes, &c->sc_prims, &c->sc_light_tri, &c->sc_light_func, &c->sc_light_cdf,
                     &c->px_seg, &c->px_keys, &c->px_keys_alt, &c->px_vals, &c->px_vals_alt, &c->px_tmp, &c->px_cls,
                     &c->chk_x, &c->chk_aux, &c->chk_y};
    for (DevMem *m : all) m->release();
    if (c->flags_host) (void)hipHostFree(c->flags_host);
    if (c->rb_host) (void)hipHostFree(c->rb_host);
    for (auto &e : c->ev)
        if (e) (void)hipEventDestroy(e);
    if (c->fork_ev) (void)hipEventDestroy(c->fork_ev);
    if (c->tile_ev) (void)hipEventDestroy(c->tile_ev);
    if (c->join_ev) (void)hipEventDestroy(c->join_ev);
    if (c->pstream) {
        (void)hipStreamSynchronize(c->pstream);
        (void)hipStreamDestroy(c->pstream);
    }
    if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char *bre_last_error(const bre_ctx *c) { return c ? c->err.c_str() : "null context"; }

bre_status bre_set_option(bre_ctx *c, int option, int64_t value) {
    if (!c) return BRE_ERR_INVALID_ARG;
    switch (option) {
    case BRE_OPT_COUNTERS: c->counters = value != 0; return BRE_OK;
    case BRE_OPT_TIMING: c->timing = value != 0; return BRE_OK;
    case BRE_OPT_KERNEL:
        if (value != 0 && value != 2 && value != 4 && value != 5)
            return fail(c, BRE_ERR_INVALID_ARG, "BRE_OPT_KERNEL must be 0, 2, 4 or 5 (kernels 1, 3 and 6 were removed)");
        c->kernel = (int)value;
        return BRE_OK;
    case BRE_OPT_LEAF_SIZE:
        if (value < 1 || value > 64) return fail(c, BRE_ERR_INVALID_ARG, "BRE_OPT_LEAF_SIZE must be in 1..64");
        c->leaf_size = (int)value;
        return BRE_OK;
    case BRE_OPT_SQRT_MODE:
        if (value != 0 && value != 1) return fail(c, BRE_ERR_INVALID_ARG, "BRE_OPT_SQRT_MODE must be 0 or 1");
        c->sqrt_mode = (int)value;
        return BRE_OK;
    case BRE_OPT_SPLIT:
        if (value < 1 || value > kMaxSplit || (value & (value - 1)))
            return fail(c, BRE_ERR_INVALID_ARG, "BRE_OPT_SPLIT must be a power of two in 1..%d", kMaxSplit);
        c->split = (int)value;
        return BRE_OK;
    case BRE_OPT_PREFILTER: c->prefilter = value != 0; return BRE_OK;
    case BRE_OPT_CHUNK_LEN:
        if (value < 25 || value > 100000)
            return fail(c, BRE_ERR_INVALID_ARG, "BRE_OPT_CHUNK_LEN must be in 25..100000 (units of E/100)");
        c->chunk_len = (int)value;
        return BRE_OK;
    case BRE_OPT_SORT_SEGMENTS: c->sort_segments = value != 0; return BRE_OK;
    case BRE_OPT_CHUNK_LEAF:
        if (value < 1 || value > 64) return fail(c, BRE_ERR_INVALID_ARG, "BRE_OPT_CHUNK_LEAF must be in 1..64");
        c->chunk_leaf = (int)value;
        return BRE_OK;
    case BRE_OPT_TILE_LEAF:
        if (value < 1 || value > 64) return fail(c, BRE_ERR_INVALID_ARG, "BRE_OPT_TILE_LEAF must be in 1..64");
        c->leaf2 = (int)value;
        return BRE_OK;
    case BRE_OPT_SHARD_RANK:
        if (value < 0 || value >= c->shard_count)
            return fail(c, BRE_ERR_INVALID_ARG, "BRE_OPT_SHARD_RANK must be in [0, shard count)");
        c->shard_rank = (int)value;
        return BRE_OK;
    case BRE_OPT_SHARD_BLOCK:
        if (value < 1 || value > 4096) return fail(c, BRE_ERR_INVALID_ARG, "BRE_OPT_SHARD_BLOCK must be in 1..4096");
        c->shard_block = (int)value;
        return BRE_OK;
    case BRE_OPT_SHARD_MODE:
        if (value < 0 || value > 2) return fail(c, BRE_ERR_INVALID_ARG, "BRE_OPT_SHARD_MODE must be 0, 1 or 2");
        c->shard_mode = (int)value;
        return BRE_OK;
    case BRE_OPT_FILM_CLASSES:
        if (value != 1 && value != BRE_FILM_CLASSES)
            return fail(c, BRE_ERR_INVALID_ARG, "BRE_OPT_FILM_CLASSES must be 1 or %d", BRE_FILM_CLASSES);
        c->film_classes = (int)value;
        return BRE_OK;
    case BRE_OPT_SHARD_COUNT:
        if (value < 1 || value > 65536) return fail(c, BRE_ERR_INVALID_ARG, "BRE_OPT_SHARD_COUNT must be in 1..65536");
        c->shard_count = (int)value;
        if (c->shard_rank >= c->shard_count) c->shard_rank = 0;
        return BRE_OK;
    case 101:  // internal: traversal stack entries to use, 0 = all (tests force an overflow)
        if (value < 0 || value > kStackDepth) return fail(c, BRE_ERR_INVALID_ARG, "stack cap must be in 0..%d", kStackDepth);
        c->stack_cap = (int)value;
        return BRE_OK;
    case 102:  // internal: tile kernel register budget, min waves per SIMD (sweeps)
        if (value != 1 && (value < 4 || value > 8))
            return fail(c, BRE_ERR_INVALID_ARG, "occupancy must be 1 or 4..8");
        c->occupancy = (int)value;
        return BRE_OK;
    case 105:  // internal: segment sort key (SegSort::key_mode, sweeps)
        if (value < 0 || value > 4) return fail(c, BRE_ERR_INVALID_ARG, "segment sort key must be 0..4");
        c->sort_key = (int)value;
        return BRE_OK;
    case 110:  // internal: tree order (1 (start, end) Morton, default; 2 the same in Hilbert order; 0 centroid)
        if (value < 0 || value > 2) return fail(c, BRE_ERR_INVALID_ARG, "tree order must be 0..2");
        c->beam_key = (int)value;
        return BRE_OK;
    case 109:  // internal: tile kernel partial-sum bytes per launch, in MiB (tests force several launches)
        if (value < 1 || value > ((int64_t)1 << 20)) return fail(c, BRE_ERR_INVALID_ARG, "partial cap must be in 1..2^20 MiB");
        c->partial_cap = value << 20;
        return BRE_OK;
    case 107:  // internal: tile kernel block mapping, 0 XCD-aware subtrees / 1 rotated / 3 LPT (sweeps)
        if (value < 0 || value > 3) return fail(c, BRE_ERR_INVALID_ARG, "block map must be 0..3");
        c->block_map = (int)value;
        return BRE_OK;
    case 108:  // internal: transposed-scan threshold in eighths, 0 = off, -1 = by MaxDistance (default; sweeps)
        if (value < -1 || value > 64) return fail(c, BRE_ERR_INVALID_ARG, "transposed-scan threshold must be in -1..64");
        c->tscan = (int)value;  // -1: by MaxDistance (tscan_for)
        return BRE_OK;
    case 112:  // internal: per-lane tile line reject, 1 on (default) / 0 off (A/B); 2 = 1 (round-4 scripts)
        if (value < 0 || value > 2) return fail(c, BRE_ERR_INVALID_ARG, "tile axis mode must be 0, 1 or 2");
        c->tile_axis = (int)value;
        return BRE_OK;
    case 113:  // internal: beam record layout, 0 power in the record for uniform-radius sets (default)
               // / 1 always radius in the record, power apart (A/B; applies from the next build)
        if (value < 0 || value > 1) return fail(c, BRE_ERR_INVALID_ARG, "record layout must be 0 or 1");
        c->split_records = (int)value;
        return BRE_OK;
    case 114:  // internal: film accumulation, 1 deterministic per-pixel compose (default) / 0 float atomics (A/B)
        if (value != 0 && value != 1) return fail(c, BRE_ERR_INVALID_ARG, "film mode must be 0 or 1");
        c->film_compose = (int)value;
        return BRE_OK;
    case 116:  // internal: photon pass, 1 single trace with per-photon slots (default) / 0 two traces (A/B) /
               // 2..64 single trace with that many slots per photon (tests: forces the overflow re-trace)
        if (value < 0 || value > 64) return fail(c, BRE_ERR_INVALID_ARG, "photon pass mode must be in 0..64");
        c->photon_single = (int)value;
        return BRE_OK;
    case 117:  // internal: photon / camera passes on a high-priority stream, 1 (default) / 0 on the caller's (A/B)
        if (value < 0 || value > 1) return fail(c, BRE_ERR_INVALID_ARG, "pass priority must be 0 or 1");
        c->pass_priority = (int)value;
        return BRE_OK;
    case 118:  // internal: small device-to-host reads by a one-wave kernel into pinned memory (1) / hipMemcpyAsync (0)
        if (value < 0 || value > 1) return fail(c, BRE_ERR_INVALID_ARG, "readback mode must be 0 or 1");
        c->kernel_readback = (int)value;
        return BRE_OK;
    case 121:  // internal: coarse sort keys (1: the tree-order sort on bits [16, 64), the segment sort on
               // [12, 60): 6 radix passes each instead of 8) / all bits (0, default)
        if (value < 0 || value > 1) return fail(c, BRE_ERR_INVALID_ARG, "coarse keys mode must be 0 or 1");
        c->coarse_keys = (int)value;
        return BRE_OK;
    case 119:  // internal: pass-chain scans / sorts / fills, 1 one-wave primitives (default) / 0 rocPRIM (A/B)
        if (value < 0 || value > 1) return fail(c, BRE_ERR_INVALID_ARG, "pass primitives mode must be 0 or 1");
        c->slot_passes = (int)value;
        return BRE_OK;
    case 111:  // internal: tile kernel prefilter margins, 1 tight (default) / 0 round 2's (A/B)
        if (value < 0 || value > 1) return fail(c, BRE_ERR_INVALID_ARG, "margin mode must be 0 or 1");
        c->margin = (int)value;
        return BRE_OK;
    default: return fail(c, BRE_ERR_INVALID_ARG, "unknown option %d", option);
    }
}

bre_status bre_set_stream(bre_ctx *c, void *stream) {
    if (!c) return BRE_ERR_INVALID_ARG;
    if (c->own_stream && c->stream) {
        (void)hipStreamSynchronize(c->stream);
        (void)hipStreamDestroy(c->stream);
    }
    if (stream) {
        c->stream = (hipStream_t)stream;
        c->own_stream = false;
    } else {
        if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)
            return fail(c, BRE_ERR_HIP, "hipStreamCreate failed");
        c->own_stream = true;
    }
    return BRE_OK;
}

bre_status bre_synchronize(bre_ctx *c) {
    if (!c) return BRE_ERR_INVALID_ARG;
    return check_flags(c);
}

bre_status bre_get_stats(const bre_ctx *c, bre_stats *out) {
    if (!c || !out) return BRE_ERR_INVALID_ARG;
    *out = c->stats;
    return BRE_OK;
}

bre_status bre_set_beams(bre_ctx *c, int64_t n, const float *start, const float *end, const float *radius,
                         const float *power) {
    if (!c) return BRE_ERR_INVALID_ARG;
    if (n < 0) return fail(c, BRE_ERR_INVALID_ARG, "bre_set_beams: negative count");
    if (n > 0 && (!start || !end || !radius || !power))
        return fail(c, BRE_ERR_INVALID_ARG, "bre_set_beams: null array");
    bre_status st = set_device(c);
    if (st != BRE_OK) return st;
    const size_t N = (size_t)n;
    if (n > 0) {
        HIPCHK(c, c->in_start.ensure(N * 3 * sizeof(float)));
        HIPCHK(c, c->in_end.ensure(N * 3 * sizeof(float)));
        HIPCHK(c, c->in_radius.ensure(N * sizeof(float)));
        HIPCHK(c, c->in_power.ensure(N * 3 * sizeof(float)));
        HIPCHK(c, hipMemcpyAsync(c->in_start.ptr, start, N * 3 * sizeof(float), hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipMemcpyAsync(c->in_end.ptr, end, N * 3 * sizeof(float), hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipMemcpyAsync(c->in_radius.ptr, radius, N * sizeof(float), hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipMemcpyAsync(c->in_power.ptr, power, N * 3 * sizeof(float), hipMemcpyHostToDevice, c->stream));
    }
    c->beams_kept = false;
    st = build(c, n, c->in_start.as<float>(), c->in_end.as<float>(), c->in_radius.as<float>(),
               c->in_power.as<float>());
    if (st != BRE_OK) return st;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->beams_kept = true;
    return BRE_OK;
}

bre_status bre_set_beams_device(bre_ctx *c, int64_t n, const float *start, const float *end, const float *radius,
                                const float *power) {
    if (!c) return BRE_ERR_INVALID_ARG;
    if (n < 0) return fail(c, BRE_ERR_INVALID_ARG, "bre_set_beams_device: negative count");
    if (n > 0 && (!start || !end || !radius || !power))
        return fail(c, BRE_ERR_INVALID_ARG, "bre_set_beams_device: null array");
    bre_status st = set_device(c);
    if (st != BRE_OK) return st;
    c->beams_kept = false;
    return build(c, n, start, end, radius, power);
}

// Medium parameters: GridDensityMedium needs a density grid with a positive maximum (the ctor's
// invMaxDensity = 1/maxDensity, grid.h:73-76); a non-uniform sigma_t is accepted as pbrt does
// (its Error() only reports it, grid.h:66-70) and channel 0 is used.
static bre_status check_medium(bre_ctx *c, const bre_scene *scene, const char *fn) {
    if (!scene) return fail(c, BRE_ERR_INVALID_ARG, "%s: null scene", fn);
    if (scene->has_medium < BRE_MEDIUM_NONE || scene->has_medium > BRE_MEDIUM_GRID)
        return fail(c, BRE_ERR_INVALID_ARG, "%s: unknown medium type %d", fn, scene->has_medium);
    if (scene->has_medium != BRE_MEDIUM_GRID) return BRE_OK;
    const int64_t nx = scene->grid_n[0], ny = scene->grid_n[1], nz = scene->grid_n[2];
    if (nx < 1 || ny < 1 || nz < 1 || nx * ny * nz > BRE_MAX_GRID_CELLS)
        return fail(c, BRE_ERR_INVALID_ARG, "%s: grid dimensions must be >= 1 with at most %d cells", fn,
                    BRE_MAX_GRID_CELLS);
    if (!scene->grid_density) return fail(c, BRE_ERR_INVALID_ARG, "%s: null grid_density", fn);
    if (!(grid_max_density(scene) > 0))
        return fail(c, BRE_ERR_INVALID_ARG, "%s: grid density maximum must be > 0", fn);
    return BRE_OK;
}

// Triangle count in range and at least one area light (the passes need scene.lights non-empty)
static bre_status check_scene(bre_ctx *c, const bre_scene *scene, const char *fn) {
    if (!scene) return fail(c, BRE_ERR_INVALID_ARG, "%s: null scene", fn);
    const int cap = scene->triangles_ext ? BRE_MAX_SCENE_TRIANGLES : BRE_MAX_TRIANGLES;
    if (scene->n_triangles < 1 || scene->n_triangles > cap)
        return fail(c, BRE_ERR_INVALID_ARG, "%s: triangle count must be in 1..%d (%s)", fn, cap,
                    scene->triangles_ext ? "triangles_ext" : "inline triangles; use triangles_ext for more");
    const bre_triangle *tri = scene_triangles(scene);
    int64_t lights = 0;
    for (int i = 0; i < scene->n_triangles; ++i) lights += tri[i].emit != 0;
    if (lights == 0) return fail(c, BRE_ERR_INVALID_ARG, "%s: the scene has no area light", fn);
    return BRE_OK;
}

// 64-bit hash of the scene's triangles (the geometry cache key of upload_scene)
static uint64_t hash_triangles(const bre_scene *s) {
    const bre_triangle *tri = scene_triangles(s);
    const size_t bytes = (size_t)s->n_triangles * sizeof(bre_triangle);
    const unsigned char *p = reinterpret_cast<const unsigned char *>(tri);
    uint64_t h = 0x9e3779b97f4a7c15ull ^ (uint64_t)s->n_triangles;
    size_t i = 0;
    for (; i + 8 <= bytes; i += 8) {
        uint64_t w;
        memcpy(&w, p + i, 8);
        h = (h ^ w) * 0x100000001b3ull;
        h ^= h >> 29;
    }
    for (; i < bytes; ++i) h = (h ^ p[i]) * 0x100000001b3ull;
    return h | 1ull;  // never 0 (= no scene)
}

// DevScene (+ the density grid of a GridDensityMedium) into ph_scene on the context's stream.  The
// geometry (triangles, BVHAccel, lights) is rebuilt and uploaded only when the triangles change.
static bre_status upload_scene(bre_ctx *c, const bre_scene *scene) {
    const float *dd = nullptr;
    if (scene->has_medium == BRE_MEDIUM_GRID) {
        const size_t n = (size_t)scene->grid_n[0] * scene->grid_n[1] * scene->grid_n[2];
        // uploaded only when the density values change (every pass of a render shares one grid)
        const unsigned char *src = reinterpret_cast<const unsigned char *>(scene->grid_density);
        const bool same = c->grid_dens.ptr && c->grid_bytes.size() == n * sizeof(float) &&
                          memcmp(c->grid_bytes.data(), src, n * sizeof(float)) == 0;
        if (!same) {
            HIPCHK(c, c->grid_dens.ensure(n * sizeof(float)));
            HIPCHK(c, hipMemcpyAsync(c->grid_dens.ptr, scene->grid_density, n * sizeof(float), hipMemcpyHostToDevice,
                                     c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
            c->grid_bytes.assign(src, src + n * sizeof(float));
        }
        dd = c->grid_dens.as<float>();
    }
    const uint64_t h = hash_triangles(scene);
    // the geometry is reused only when the hash AND the bytes match (a hash collision between two
    // scenes must not trace against the stale BVH and lights)
    const size_t tri_bytes = (size_t)scene->n_triangles * sizeof(bre_triangle);
    const bool same = h == c->sc_hash && c->sc_bytes.size() == tri_bytes &&
                      (tri_bytes == 0 || memcmp(c->sc_bytes.data(), scene_triangles(scene), tri_bytes) == 0);
    if (!same) {
        HostScene hs;
        prepare_geometry(scene, &hs);
        if (hs.depth > kSceneStack)
            return fail(c, BRE_ERR_INVALID_ARG, "scene BVH depth %d exceeds the %d-entry traversal stack (as in "
                        "BVHAccel::Intersect)", hs.depth, kSceneStack);
        const auto up = [&](DevMem &m, const void *src, size_t bytes) -> hipError_t {
            hipError_t e = m.ensure(bytes > 0 ? bytes : 4);
            if (e != hipSuccess || bytes == 0) return e;
            return hipMemcpyAsync(m.ptr, src, bytes, hipMemcpyHostToDevice, c->stream);
        };
        HIPCHK(c, up(c->sc_tris, hs.tris.data(), hs.tris.size() * sizeof(PTri)));
        HIPCHK(c, up(c->sc_nodes, hs.nodes.data(), hs.nodes.size() * sizeof(SceneNode)));
        HIPCHK(c, up(c->sc_prims, hs.prims.data(), hs.prims.size() * sizeof(int32_t)));
        HIPCHK(c, up(c->sc_light_tri, hs.light_tri.data(), hs.light_tri.size() * sizeof(int32_t)));
        HIPCHK(c, up(c->sc_light_func, hs.light_func.data(), hs.light_func.size() * sizeof(float)));
        HIPCHK(c, up(c->sc_light_cdf, hs.light_cdf.data(), hs.light_cdf.size() * sizeof(float)));
        HIPCHK(c, hipStreamSynchronize(c->stream));  // the host vectors go out of scope
        c->sc_head = hs.head;
        c->sc_head.t = c->sc_tris.as<PTri>();
        c->sc_head.nodes = c->sc_nodes.as<SceneNode>();
        c->sc_head.prims = c->sc_prims.as<int32_t>();
        c->sc_head.light_tri = c->sc_light_tri.as<int32_t>();
        c->sc_head.light_func = c->sc_light_func.as<float>();
        c->sc_head.light_cdf = c->sc_light_cdf.as<float>();
        c->sc_hash = h;
        const unsigned char *tb = reinterpret_cast<const unsigned char *>(scene_triangles(scene));
        c->sc_bytes.assign(tb, tb + tri_bytes);
    }
    DevScene ds;
    memcpy(&ds, &c->sc_head, sizeof(DevScene));  // padding bytes included: the record compares bytewise
    prepare_medium(scene, &ds, dd);
    // the scene record is copied only when it changes: in a render every pass uploads the same record,
    // and a copy queued behind another context's gather waits for that gather's blocks (round 5 trace:
    // a 1.6 KB upload took 110 ms in the two-context pipeline)
    if (!c->ph_scene.ptr || memcmp(&ds, &c->ph_scene_host, sizeof(DevScene)) != 0) {
        HIPCHK(c, c->ph_scene.ensure(sizeof(DevScene)));
        HIPCHK(c, hipMemcpyAsync(c->ph_scene.ptr, &ds, sizeof(DevScene), hipMemcpyHostToDevice, c->stream));
        // the host copies are read by the DMA before the call returns
        HIPCHK(c, hipStreamSynchronize(c->stream));
        memcpy(&c->ph_scene_host, &ds, sizeof(DevScene));
    }
    return BRE_OK;
}

bre_status bre_trace_photons(bre_ctx *c, const bre_scene *scene, int64_t n_photons, int32_t iteration,
                             int32_t max_depth, float beam_radius, int64_t *n_beams) {
    if (!c) return BRE_ERR_INVALID_ARG;
    if (n_beams) *n_beams = 0;
    if (!scene) return fail(c, BRE_ERR_INVALID_ARG, "bre_trace_photons: null scene");
    if (n_photons < 0 || iteration < 0) return fail(c, BRE_ERR_INVALID_ARG, "bre_trace_photons: negative count");
    if (max_depth < 1 || max_depth > BRE_MAX_DEPTH)
        return fail(c, BRE_ERR_INVALID_ARG, "bre_trace_photons: max_depth must be in [1, %d]", BRE_MAX_DEPTH);
    bre_status st = check_scene(c, scene, "bre_trace_photons");
    if (st != BRE_OK) return st;
    st = check_medium(c, scene, "bre_trace_photons");
    if (st != BRE_OK) return st;
    st = set_device(c);
    if (st != BRE_OK) return st;
    PassStream pass(c);
    // an earlier asynchronous gather's device errors are reported before this call changes anything
    st = check_flags(c);
    if (st != BRE_OK) return st;
    st = upload_scene(c, scene);
    if (st != BRE_OK) return st;
    const size_t N = (size_t)n_photons;
    HIPCHK(c, c->ph_counts.ensure((N + 1) * sizeof(int32_t)));
    HIPCHK(c, c->ph_offsets.ensure((N + 1) * sizeof(int64_t)));
    const size_t tmp = count_scan_temp_bytes(n_photons);
    HIPCHK(c, c->ph_tmp.ensure(tmp + 16));
    const uint64_t seq0 = (uint64_t)iteration * (uint64_t)n_photons + 1;
    const DevScene *ds = c->ph_scene.as<DevScene>();
    if (c->timing) HIPCHK(c, hipEventRecord(c->ev[0], c->stream));
    const int sdepth = c->sc_head.stack_depth;
    // single-trace form (bre_photon.hip): `cap` beam slots per photon, scratch at most 2.5 GB (62 slots at
    // 1M photons: the re-trace of the photons with more beams than slots is the form's tail, 1.65 ms
    // with 16 slots vs 1.41 with 64 at C2, profiles/r4/run36); below 4 slots, or with option 116 = 0,
    // the two-trace form
    int cap = c->photon_single ? (int)std::min<int64_t>(64, ((int64_t)5 << 29) / (40 * std::max<int64_t>(n_photons, 1))) : 0;
    if (cap < 4) cap = 0;
    if (c->photon_single >= 2) cap = c->photon_single;  // tests: a forced slot count (overflow paths)
    if (cap > 0) {
        const size_t slots = N * (size_t)cap;
        HIPCHK(c, c->ph_s_start.ensure(slots * 3 * sizeof(float)));
        HIPCHK(c, c->ph_s_end.ensure(slots * 3 * sizeof(float)));
        HIPCHK(c, c->ph_s_radius.ensure(slots * sizeof(float)));
        HIPCHK(c, c->ph_s_power.ensure(slots * 3 * sizeof(float)));
        HIPCHK(c, launch_photons(ds, sdepth, n_photons, seq0, max_depth, beam_radius, c->ph_counts.as<int32_t>(),
                                 nullptr, c->ph_s_start.as<float>(), c->ph_s_end.as<float>(), c->ph_s_radius.as<float>(),
                                 c->ph_s_power.as<float>(), 2, cap, c->stream));
    } else {
        HIPCHK(c, launch_photons(ds, sdepth, n_photons, seq0, max_depth, beam_radius, c->ph_counts.as<int32_t>(),
                                 nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0, c->stream));
    }
    HIPCHK(c, launch_count_scan(c->ph_tmp.ptr, c->ph_tmp.cap, c->ph_counts.as<int32_t>(), c->ph_offsets.as<int64_t>(),
                                n_photons, c->stream, c->slot_passes != 0));
    int64_t total = 0;
    st = read_small(c, {{&total, c->ph_offsets.as<int64_t>() + n_photons, sizeof(total)}});
    if (st != BRE_OK) return st;
    const size_t B = (size_t)total;
    if (total > 0) {
        HIPCHK(c, c->in_start.ensure(B * 3 * sizeof(float)));
        HIPCHK(c, c->in_end.ensure(B * 3 * sizeof(float)));
        HIPCHK(c, c->in_radius.ensure(B * sizeof(float)));
        HIPCHK(c, c->in_power.ensure(B * 3 * sizeof(float)));
        if (cap > 0)
            HIPCHK(c, launch_photon_slots(n_photons, cap, c->ph_counts.as<int32_t>(), c->ph_offsets.as<int64_t>(),
                                          c->ph_s_start.as<float>(), c->ph_s_end.as<float>(), c->ph_s_radius.as<float>(),
                                          c->ph_s_power.as<float>(), c->in_start.as<float>(), c->in_end.as<float>(),
                                          c->in_radius.as<float>(), c->in_power.as<float>(), c->stream));
        // every photon (two-trace form), or only those with more beams than slots
        HIPCHK(c, launch_photons(ds, sdepth, n_photons, seq0, max_depth, beam_radius, c->ph_counts.as<int32_t>(),
                                 c->ph_offsets.as<int64_t>(), c->in_start.as<float>(), c->in_end.as<float>(),
                                 c->in_radius.as<float>(), c->in_power.as<float>(), 1, cap, c->stream));
    }
    float photon_ms = 0.f;
    if (c->timing) {
        HIPCHK(c, hipEventRecord(c->ev[1], c->stream));
        HIPCHK(c, hipEventSynchronize(c->ev[1]));
        HIPCHK(c, hipEventElapsedTime(&photon_ms, c->ev[0], c->ev[1]));
    }
    c->beams_kept = false;
    st = build(c, total, c->in_start.as<float>(), c->in_end.as<float>(), c->in_radius.as<float>(),
               c->in_power.as<float>());
    if (st != BRE_OK) return st;
    c->beams_kept = true;
    c->stats.n_photons = n_photons;
    c->stats.photon_ms = photon_ms;
    if (n_beams) *n_beams = total;
    return check_flags(c);
}

bre_status bre_get_beams(bre_ctx *c, int64_t capacity, float *start, float *end, float *radius, float *power,
                         int64_t *n_beams) {
    if (!c) return BRE_ERR_INVALID_ARG;
    if (capacity < 0) return fail(c, BRE_ERR_INVALID_ARG, "bre_get_beams: negative capacity");
    if (!c->beams_kept && c->nbeams > 0)
        return fail(c, BRE_ERR_STATE, "bre_get_beams: the beam set came from caller device arrays");
    if (n_beams) *n_beams = c->nbeams;
    const int64_t k = capacity < c->nbeams ? capacity : c->nbeams;
    if (k <= 0) return BRE_OK;
    if (!start || !end || !radius || !power) return fail(c, BRE_ERR_INVALID_ARG, "bre_get_beams: null array");
    bre_status st = set_device(c);
    if (st != BRE_OK) return st;
    const size_t K = (size_t)k;
    HIPCHK(c, hipMemcpyAsync(start, c->in_start.ptr, K * 3 * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(end, c->in_end.ptr, K * 3 * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(radius, c->in_radius.ptr, K * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(power, c->in_power.ptr, K * 3 * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    return check_flags(c);
}



bre_status bre_camera_pass(bre_ctx *c, const bre_scene *scene, int32_t width, int32_t height, int32_t iteration,
                           int32_t max_depth, int32_t render_surfaces, int32_t render_media, float *d_surface,
                           int64_t *n_segments) {
    if (!c) return BRE_ERR_INVALID_ARG;
    if (n_segments) *n_segments = 0;
    bre_status st = check_scene(c, scene, "bre_camera_pass");
    if (st != BRE_OK) return st;
    if (width < 1 || height < 1 || (int64_t)width * height > (int64_t)INT32_MAX / BRE_MAX_DEPTH || iteration < 0)
        return fail(c, BRE_ERR_INVALID_ARG, "bre_camera_pass: bad film size or iteration");
    if (max_depth < 1 || max_depth > BRE_MAX_DEPTH)
        return fail(c, BRE_ERR_INVALID_ARG, "bre_camera_pass: max_depth must be in [1, %d]", BRE_MAX_DEPTH);
    st = check_medium(c, scene, "bre_camera_pass");
    if (st != BRE_OK) return st;
    st = set_device(c);
    if (st != BRE_OK) return st;
    PassStream pass(c);
    st = check_flags(c);  // an earlier gather's device errors, before this pass changes anything
    if (st != BRE_OK) return st;
    // scene + camera/Halton tables (rebuilt when the scene or film changes)
    st = upload_scene(c, scene);
    if (st != BRE_OK) return st;
    if (c->cam_w != width || c->cam_h != height || memcmp(&c->cam_scene, scene, sizeof(bre_scene)) != 0) {
        DevCamera cam;
        std::vector<uint16_t> perms;
        prepare_camera(scene, width, height, &cam, &perms);
        HIPCHK(c, c->cam_dev.ensure(sizeof(DevCamera)));
        HIPCHK(c, c->cam_perms.ensure(perms.size() * sizeof(uint16_t)));
        HIPCHK(c, hipMemcpyAsync(c->cam_dev.ptr, &cam, sizeof(cam), hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipMemcpyAsync(c->cam_perms.ptr, perms.data(), perms.size() * sizeof(uint16_t),
                                 hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));  // host vectors go out of scope
        c->cam_w = width;
        c->cam_h = height;
        memcpy(&c->cam_scene, scene, sizeof(bre_scene));
    }
    const int64_t nslots = camera_slots(width, height);
    const size_t S = (size_t)(nslots * max_depth);
    HIPCHK(c, c->cs_o.ensure(S * 3 * sizeof(float)));
    HIPCHK(c, c->cs_p.ensure(S * 3 * sizeof(float)));
    HIPCHK(c, c->cs_d.ensure(S * 3 * sizeof(float)));
    HIPCHK(c, c->cs_t.ensure(S * sizeof(float)));
    HIPCHK(c, c->cs_pix.ensure(S * sizeof(int32_t)));
    HIPCHK(c, c->cs_valid.ensure(S * sizeof(int32_t)));
    HIPCHK(c, c->cam_offs.ensure((S + 1) * sizeof(int64_t)));
    const size_t tmp = camera_scan_temp_bytes((int64_t)S);
    HIPCHK(c, c->cam_tmp.ensure(tmp + 16));
    HIPCHK(c, c->cam_flags.ensure(sizeof(unsigned int)));
    HIPCHK(c, fill_words(c, c->cam_flags.ptr, sizeof(unsigned int)));
    CamSlots cs{c->cs_o.as<float>(), c->cs_p.as<float>(), c->cs_d.as<float>(), c->cs_t.as<float>(),
                c->cs_pix.as<int32_t>(), c->cs_valid.as<int32_t>()};
    if (c->timing) HIPCHK(c, hipEventRecord(c->ev[0], c->stream));
    HIPCHK(c, launch_camera(c->ph_scene.as<DevScene>(), c->sc_head.stack_depth, c->cam_dev.as<DevCamera>(),
                            c->cam_perms.as<uint16_t>(),
                            width, height, iteration, max_depth, render_surfaces, render_media, cs, d_surface,
                            c->cam_flags.as<unsigned int>(), c->shard_rank, c->shard_count,
                            c->shard_mode != 0 ? 0 : c->shard_block, c->film_classes, c->stream));
    // total = offs[S-1] + valid[S-1]
    HIPCHK(c, rocprim_free_total_scan(c, cs, nslots, max_depth));
    int64_t last_off = 0;
    int32_t last_valid = 0;
    unsigned int flags = 0;
    st = read_small(c, {{&last_off, c->cam_offs.as<int64_t>() + (S - 1), sizeof(int64_t)},
                        {&last_valid, c->cs_valid.as<int32_t>() + (S - 1), sizeof(int32_t)},
                        {&flags, c->cam_flags.ptr, sizeof(flags)}});
    if (st != BRE_OK) return st;
    const int64_t n = last_off + last_valid;
    const size_t N = (size_t)(n > 0 ? n : 1);
    HIPCHK(c, c->seg_o.ensure(N * 3 * sizeof(float)));
    HIPCHK(c, c->seg_p.ensure(N * 3 * sizeof(float)));
    HIPCHK(c, c->seg_d.ensure(N * 3 * sizeof(float)));
    HIPCHK(c, c->seg_t.ensure(N * sizeof(float)));
    HIPCHK(c, c->seg_pix.ensure(N * sizeof(int32_t)));
    HIPCHK(c, c->seg_depth.ensure(N * sizeof(int32_t)));
    HIPCHK(c, launch_camera_compact(cs, nslots, max_depth, c->cam_offs.as<int64_t>(), c->seg_o.as<float>(),
                                    c->seg_p.as<float>(), c->seg_d.as<float>(), c->seg_t.as<float>(),
                                    c->seg_pix.as<int32_t>(), c->seg_depth.as<int32_t>(), c->stream));
    float ms = 0.f;
    if (c->timing) {
        HIPCHK(c, hipEventRecord(c->ev[1], c->stream));
        HIPCHK(c, hipEventSynchronize(c->ev[1]));
        HIPCHK(c, hipEventElapsedTime(&ms, c->ev[0], c->ev[1]));
    }
    c->cam_nseg = n;
    c->cam_npix = (int64_t)width * height;
    c->stats.n_camera_segments = n;
    c->stats.camera_ms = ms;
    if (n_segments) *n_segments = n;
    return check_flags(c);
}

// n device segments against the beam set in the production order: the segments only add into
// their pixels, so the packet kernel takes them in a coherence order (bre_sort.hip; kernels 0 / 4);
// per-segment outputs (optional) are scattered back to the caller's order.  Under
// BRE_OPT_SHARD_MODE 1 with a shard count > 1 only this shard's packets of that order are gathered
// (bre_shard_segments): the other entries of the per-segment outputs are zeroed, and the shards'
// films and outputs sum to the one-shard results.  Used by bre_gather_camera (the camera pass's
// segments), bre_gather_device and bre_gather (the caller's segments).
static bre_status gather_segments_core(bre_ctx *c, int64_t n, const float *o, const float *p, const float *d,
                                       const float *t, const int32_t *pix, float R, int64_t npix, float *d_accum,
                                       float *d_seg_rgb, int32_t *d_seg_counts) {
    const bool pshard = c->shard_mode == 1 && c->shard_count > 1;
    const bool sortable = c->kernel == 0 || c->kernel == 4;  // kernels 2 / 5 write in the caller's order
    const bool seg_out = d_seg_rgb || d_seg_counts;
    if (n < 0 || npix < 0) return fail(c, BRE_ERR_INVALID_ARG, "bre_gather: negative size");
    if (n > 0 && (!o || !p || !d || !t)) return fail(c, BRE_ERR_INVALID_ARG, "bre_gather: null segment array");
    if (d_accum && !pix) return fail(c, BRE_ERR_INVALID_ARG, "bre_gather: accum_rgb given without seg_pixel");
    if (pshard && seg_out) {
        if (!sortable) return fail(c, BRE_ERR_STATE, "packet shards with per-segment outputs need kernel 0 or 4");
        // every entry is defined: the other shards' segments read 0 here
        GatherArgs z{};
        z.nseg = n;
        z.seg_rgb = d_seg_rgb;
        z.seg_counts = d_seg_counts;
        HIPCHK(c, launch_zero_outputs(z, c->stream));
    }
    // packet sharding: this shard gathers the chunks c = rank (mod count) of BRE_OPT_SHARD_BLOCK
    // consecutive 64-segment packets of the (sorted) order, copied into contiguous arrays first
    const auto pick = [&](const float *o, const float *p, const float *d, const float *t, const int32_t *pix,
                          const int32_t *index) -> bre_status {
        const int64_t m = bre_shard_segments(n, c->shard_rank, c->shard_count, c->shard_block);
        c->stats.n_segments = m;
        if (m == 0) return BRE_OK;
        const size_t M = (size_t)m;
        HIPCHK(c, c->sp_o.ensure(M * 3 * sizeof(float)));
        HIPCHK(c, c->sp_p.ensure(M * 3 * sizeof(float)));
        HIPCHK(c, c->sp_d.ensure(M * 3 * sizeof(float)));
        HIPCHK(c, c->sp_t.ensure(M * sizeof(float)));
        HIPCHK(c, c->sp_pix.ensure(M * sizeof(int32_t)));
        if (seg_out) HIPCHK(c, c->sp_index.ensure(M * sizeof(int32_t)));
        HIPCHK(c, launch_packet_pick(n, m, c->shard_rank, c->shard_count, c->shard_block, o, p, d, t, pix, index,
                                     c->sp_o.as<float>(), c->sp_p.as<float>(), c->sp_d.as<float>(),
                                     c->sp_t.as<float>(), c->sp_pix.as<int32_t>(),
                                     seg_out ? c->sp_index.as<int32_t>() : nullptr, c->stream));
        return gather_device(c, m, c->sp_o.as<float>(), c->sp_p.as<float>(), c->sp_d.as<float>(),
                             c->sp_t.as<float>(), pix ? c->sp_pix.as<int32_t>() : nullptr, R, npix, d_accum,
                             d_seg_rgb, d_seg_counts, seg_out ? c->sp_index.as<int32_t>() : nullptr);
    };
    if (!c->sort_segments || n < 2 || (!sortable && seg_out)) {
        if (pshard) return pick(o, p, d, t, pix, nullptr);
        return gather_device(c, n, o, p, d, t, pix, R, npix, d_accum, d_seg_rgb, d_seg_counts);
    }
    const size_t N = (size_t)n;
    HIPCHK(c, c->ss_bounds.ensure(8 * sizeof(unsigned int)));
    HIPCHK(c, c->ss_keys.ensure(N * sizeof(unsigned long long)));
    HIPCHK(c, c->ss_keys_alt.ensure(N * sizeof(unsigned long long)));
    HIPCHK(c, c->ss_vals.ensure(N * sizeof(int32_t)));
    HIPCHK(c, c->ss_vals_alt.ensure(N * sizeof(int32_t)));
    const size_t tb = seg_sort_temp_bytes(n);
    HIPCHK(c, c->ss_tmp.ensure(tb + 16));
    HIPCHK(c, c->ss_o.ensure(N * 3 * sizeof(float)));
    HIPCHK(c, c->ss_p.ensure(N * 3 * sizeof(float)));
    HIPCHK(c, c->ss_d.ensure(N * 3 * sizeof(float)));
    HIPCHK(c, c->ss_t.ensure(N * sizeof(float)));
    HIPCHK(c, c->ss_pix.ensure(N * sizeof(int32_t)));
    SegSort ss{n, o, p, d, t, pix, c->ss_bounds.as<unsigned int>(), c->ss_keys.as<unsigned long long>(),
               c->ss_keys_alt.as<unsigned long long>(), c->ss_vals.as<int32_t>(), c->ss_vals_alt.as<int32_t>(),
               c->ss_tmp.ptr, tb, c->ss_o.as<float>(), c->ss_p.as<float>(), c->ss_d.as<float>(),
               c->ss_t.as<float>(), c->ss_pix.as<int32_t>(), c->sort_key, c->slot_passes, c->coarse_keys ? 12 : 0};
    HIPCHK(c, launch_sort_segments(ss, c->stream));
    // ss_vals_alt[i] = the caller's index of sorted segment i (the sort's permutation)
    if (pshard) return pick(ss.o2, ss.p2, ss.d2, ss.t2, ss.pix2, c->ss_vals_alt.as<int32_t>());
    return gather_device(c, n, ss.o2, ss.p2, ss.d2, ss.t2, pix ? ss.pix2 : nullptr, R, npix, d_accum, d_seg_rgb,
                         d_seg_counts, seg_out ? c->ss_vals_alt.as<int32_t>() : nullptr);
}

// A gather of n caller-order segments.  With a film (d_accum) the production kernels (0 / 4) add to it
// deterministically: the per-segment sums go to a buffer in the caller's order (the caller's d_seg_rgb
// or an internal one; under packet shards the other shards' entries are 0), then launch_pixel_compose
// adds each pixel's segments in the caller's order -- for the camera pass, the path depths in order,
// as the reference's pixel.Ld += does (photonbeam.cpp:477-504) -- with one thread per pixel and no
// float atomics, so the film is the same bits on every run.  Kernels 2 and 5 (cross-checks) add by
// float atomics.
static bre_status gather_segments(bre_ctx *c, int64_t n, const float *o, const float *p, const float *d,
                                  const float *t, const int32_t *pix, float R, int64_t npix, float *d_accum,
                                  float *d_seg_rgb, int32_t *d_seg_counts) {
    const bool sortable = c->kernel == 0 || c->kernel == 4;
    if (c->film_classes > 1 && d_accum && (!sortable || !c->film_compose))
        return fail(c, BRE_ERR_STATE, "BRE_OPT_FILM_CLASSES needs the deterministic compose of kernels 0 / 4");
    // work-root shards gather every segment against a subset of the subtrees: each rank's sums are partial in
    // every class plane, so per-rank planes cannot be gathered plane by plane (dist.ShardedFrame refuses it too)
    if (c->film_classes > 1 && d_accum && c->shard_mode == 2 && c->shard_count > 1)
        return fail(c, BRE_ERR_STATE, "BRE_OPT_FILM_CLASSES needs packet shards (BRE_OPT_SHARD_MODE 1), not work-root shards");
    if (c->film_classes > 1 && d_accum && (uint64_t)BRE_FILM_CLASSES * (uint64_t)(npix + 1) > 0xffffffffull)
        return fail(c, BRE_ERR_INVALID_ARG, "BRE_OPT_FILM_CLASSES: the film is too large for the class keys");
    if (!d_accum || !sortable || n <= 0 || !pix || c->nvalid == 0 || !c->film_compose)
        return gather_segments_core(c, n, o, p, d, t, pix, R, npix, d_accum, d_seg_rgb, d_seg_counts);
    const size_t N = (size_t)n;
    float *segbuf = d_seg_rgb;
    if (!segbuf) {
        HIPCHK(c, c->px_seg.ensure(N * 3 * sizeof(float)));
        segbuf = c->px_seg.as<float>();
    }
    bre_status st = gather_segments_core(c, n, o, p, d, t, pix, R, npix, nullptr, segbuf, d_seg_counts);
    if (st != BRE_OK) return st;
    HIPCHK(c, c->px_keys.ensure(N * sizeof(unsigned int)));
    HIPCHK(c, c->px_keys_alt.ensure(N * sizeof(unsigned int)));
    HIPCHK(c, c->px_vals.ensure(N * sizeof(int32_t)));
    HIPCHK(c, c->px_vals_alt.ensure(N * sizeof(int32_t)));
    const size_t tb = pixel_sort_temp_bytes(n);
    HIPCHK(c, c->px_tmp.ensure(tb + 16));
    // the flags word of the counter block (a packet shard with no segments never reached the gather's
    // counters_block, so make sure it exists)
    if (!c->counters_buf.ptr) {
        DevCounters *fresh = nullptr;
        st = counters_block(c, &fresh);
        if (st != BRE_OK) return st;
    }
    DevCounters *ctr = c->counters_buf.as<DevCounters>();
    const uint8_t *cls = nullptr;
    if (c->film_classes > 1) {
        // each segment's class: its packet chunk in the order the gather used (sorted when sorting is on)
        HIPCHK(c, c->px_cls.ensure(N));
        const bool sorted = c->sort_segments && n >= 2;
        HIPCHK(c, launch_seg_classes(n, c->shard_block, c->film_classes, sorted ? c->ss_vals_alt.as<int32_t>() : nullptr,
                                     c->px_cls.as<uint8_t>(), c->stream));
        cls = c->px_cls.as<uint8_t>();
    }
    PixelCompose pc{n, pix, segbuf, npix, d_accum, cls, c->film_classes, c->px_keys.as<unsigned int>(),
                    c->px_keys_alt.as<unsigned int>(), c->px_vals.as<int32_t>(), c->px_vals_alt.as<int32_t>(),
                    c->px_tmp.ptr, tb, &ctr->flags, kFlagPixel, c->slot_passes};
    HIPCHK(c, launch_pixel_compose(pc, c->stream));
    return BRE_OK;
}

// The camera segments of the last camera pass against the beam set (gather_segments).
static bre_status gather_camera(bre_ctx *c, float R, float *d_accum, float *d_seg_rgb, int32_t *d_seg_counts) {
    if (c->cam_npix == 0) return fail(c, BRE_ERR_STATE, "bre_gather_camera: no camera pass yet");
    bre_status st = set_device(c);
    if (st != BRE_OK) return st;
    return gather_segments(c, c->cam_nseg, c->seg_o.as<float>(), c->seg_p.as<float>(), c->seg_d.as<float>(),
                           c->seg_t.as<float>(), c->seg_pix.as<int32_t>(), R, c->cam_npix, d_accum, d_seg_rgb,
                           d_seg_counts);
}

bre_status bre_resolve_classes(bre_ctx *c, int64_t npix, const float *d_classes, float *d_out) {
    if (!c) return BRE_ERR_INVALID_ARG;
    if (npix < 0 || (npix > 0 && (!d_classes || !d_out))) return fail(c, BRE_ERR_INVALID_ARG, "bre_resolve_classes: bad film");
    bre_status st = set_device(c);
    if (st != BRE_OK) return st;
    HIPCHK(c, launch_resolve_classes(3 * npix, BRE_FILM_CLASSES, d_classes, d_out, c->stream));
    return BRE_OK;
}

bre_status bre_set_gather_events(bre_ctx *c, void *start_event, void *end_event) {
    if (!c) return BRE_ERR_INVALID_ARG;
    c->user_ev[0] = static_cast<hipEvent_t>(start_event);
    c->user_ev[1] = static_cast<hipEvent_t>(end_event);
    return BRE_OK;
}

bre_status bre_set_gather_after(bre_ctx *c, bre_ctx *prev) {
    if (!c) return BRE_ERR_INVALID_ARG;
    if (prev == c || (prev && prev->device != c->device))
        return fail(c, BRE_ERR_INVALID_ARG, "bre_set_gather_after: another context of the same device");
    std::lock_guard<std::mutex> lk(link_mu());
    if (c->after) unlink_follower(c->after, c);
    c->after = prev;
    if (prev) prev->followers.push_back(c);
    return BRE_OK;
}

bre_status bre_film_add(bre_ctx *c, int64_t n_floats, float *d_src, float *d_dst, int32_t clear_src) {
    if (!c) return BRE_ERR_INVALID_ARG;
    if (n_floats < 0 || (n_floats > 0 && (!d_src || !d_dst)) || d_src == d_dst)
        return fail(c, BRE_ERR_INVALID_ARG, "bre_film_add: bad films");
    bre_status st = set_device(c);
    if (st != BRE_OK) return st;
    HIPCHK(c, launch_film_add(n_floats, d_src, d_dst, clear_src != 0, c->stream));
    return BRE_OK;
}

bre_status bre_gather_camera(bre_ctx *c, float R, float *d_accum) {
    if (!c) return BRE_ERR_INVALID_ARG;
    return gather_camera(c, R, d_accum, nullptr, nullptr);
}

bre_status bre_gather_camera_segments(bre_ctx *c, float R, float *d_accum, float *d_seg_rgb, int32_t *d_seg_counts) {
    if (!c) return BRE_ERR_INVALID_ARG;
    return gather_camera(c, R, d_accum, d_seg_rgb, d_seg_counts);
}

bre_status bre_get_segments(bre_ctx *c, int64_t capacity, float *o, float *p, float *d, float *tmax, int32_t *pixel,
                            int32_t *depth, int64_t *n_segments) {
    if (!c) return BRE_ERR_INVALID_ARG;
    if (capacity < 0) return fail(c, BRE_ERR_INVALID_ARG, "bre_get_segments: negative capacity");
    if (n_segments) *n_segments = c->cam_nseg;
    const int64_t k = capacity < c->cam_nseg ? capacity : c->cam_nseg;
    if (k <= 0) return BRE_OK;
    if (!o || !p || !d || !tmax || !pixel || !depth)
        return fail(c, BRE_ERR_INVALID_ARG, "bre_get_segments: null array");
    bre_status st = set_device(c);
    if (st != BRE_OK) return st;
    const size_t K = (size_t)k;
    HIPCHK(c, hipMemcpyAsync(o, c->seg_o.ptr, K * 3 * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(p, c->seg_p.ptr, K * 3 * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(d, c->seg_d.ptr, K * 3 * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(tmax, c->seg_t.ptr, K * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(pixel, c->seg_pix.ptr, K * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(depth, c->seg_depth.ptr, K * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    return check_flags(c);
}

static bre_status check_params(bre_ctx *c, const bre_render_params *rp) {
    if (!rp) return fail(c, BRE_ERR_INVALID_ARG, "bre_render: null params");
    if (rp->width < 1 || rp->height < 1 || rp->start_iteration < 0 ||
        rp->end_iteration < rp->start_iteration || rp->max_depth < 1 || rp->max_depth > BRE_MAX_DEPTH)
        return fail(c, BRE_ERR_INVALID_ARG, "bre_render: bad parameters");
    return BRE_OK;
}

bre_status bre_render_iteration(bre_ctx *c, const bre_scene *scene, const bre_render_params *rp, int32_t iteration,
                                float *d_ld) {
    if (!c) return BRE_ERR_INVALID_ARG;
    bre_status st = check_params(c, rp);
    if (st != BRE_OK) return st;
    if (!d_ld) return fail(c, BRE_ERR_INVALID_ARG, "bre_render_iteration: null Ld buffer");
    const float R = bre_beam_radius_at(rp->initial_radius, rp->alpha, iteration);
    // photonsperiteration <= 0 means the film's pixel count (photonbeam.h:37-39, the -1 default)
    const int64_t photons =
        rp->photons_per_iteration > 0 ? rp->photons_per_iteration : (int64_t)rp->width * rp->height;
    st = bre_trace_photons(c, scene, photons, iteration, rp->max_depth, R, nullptr);
    if (st != BRE_OK) return st;
    st = bre_camera_pass(c, scene, rp->width, rp->height, iteration, rp->max_depth, rp->render_surfaces,
                         rp->render_media, d_ld, nullptr);
    if (st != BRE_OK) return st;
    if (rp->render_media) return bre_gather_camera(c, R, d_ld);
    return BRE_OK;
}

bre_status bre_render_progressive(bre_ctx *c, const bre_scene *scene, const bre_render_params *rp,
                                  int32_t write_frequency, bre_image_fn on_image, void *user) {
    if (!c) return BRE_ERR_INVALID_ARG;
    bre_status st = check_params(c, rp);
    if (st != BRE_OK) return st;
    if (c->film_classes > 1) return fail(c, BRE_ERR_STATE, "bre_render*: BRE_OPT_FILM_CLASSES is for caller device films");
    st = set_device(c);
    if (st != BRE_OK) return st;
    const int64_t npix = (int64_t)rp->width * rp->height;
    float *ld = nullptr;
    HIPCHK(c, hipMalloc(&ld, (size_t)npix * 3 * sizeof(float)));
    st = BRE_OK;
    if (hipMemsetAsync(ld, 0, (size_t)npix * 3 * sizeof(float), c->stream) != hipSuccess)
        st = fail(c, BRE_ERR_HIP, "bre_render: memset failed");
    std::vector<float> h, img;
    for (int it = rp->start_iteration; st == BRE_OK && it < rp->end_iteration; ++it) {
        st = bre_render_iteration(c, scene, rp, it, ld);
        if (st != BRE_OK) break;
        // photonbeam.cpp:564: write at the last iteration and whenever (iter + 1) % writeFrequency == 0,
        // negative frequencies included (-k fires every k iterations); the reference's default
        // 1 << 31 wraps to INT32_MIN and never fires, and 0 (a division by zero there) means never
        const bool periodic = write_frequency != 0 && write_frequency != INT32_MIN &&
                              (it + 1) % write_frequency == 0;
        const bool write = (it + 1 == rp->end_iteration) || periodic;
        if (!write || !on_image) continue;
        h.resize((size_t)npix * 3);
        img.resize(h.size());
        if (hipMemcpyAsync(h.data(), ld, h.size() * sizeof(float), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
            hipStreamSynchronize(c->stream) != hipSuccess) {
            st = fail(c, BRE_ERR_HIP, "bre_render: copy-back failed");
            break;
        }
        st = bre_resolve_image(npix, h.data(), it, img.data());  // L = Ld / (iter + 1), :578
        if (st == BRE_OK && on_image(it, img.data(), user) != 0)
            st = fail(c, BRE_ERR_STATE, "bre_render: image callback stopped the render after iteration %d", it);
    }
    const bre_status fst = check_flags(c);  // the last iteration's gather
    if (st == BRE_OK) st = fst;
    (void)hipFree(ld);
    return st;
}

namespace {
struct FinalImage {
    float *dst;
    size_t n;
};
int keep_final_image(int32_t, const float *img, void *user) {
    FinalImage *f = static_cast<FinalImage *>(user);
    memcpy(f->dst, img, f->n * sizeof(float));
    return 0;
}
}  // namespace

bre_status bre_render(bre_ctx *c, const bre_scene *scene, const bre_render_params *rp, float *image) {
    if (!c) return BRE_ERR_INVALID_ARG;
    bre_status st = check_params(c, rp);
    if (st != BRE_OK) return st;
    if (c->film_classes > 1) return fail(c, BRE_ERR_STATE, "bre_render: BRE_OPT_FILM_CLASSES is for caller device films");
    if (!image) return fail(c, BRE_ERR_INVALID_ARG, "bre_render: null image");
    FinalImage f{image, (size_t)rp->width * rp->height * 3};
    if (rp->end_iteration == rp->start_iteration) {
        memset(image, 0, f.n * sizeof(float));
        return BRE_OK;
    }
    // only the last iteration's image is kept (write_frequency 0 = at the end only)
    return bre_render_progressive(c, scene, rp, 0, keep_final_image, &f);
}

void bre_scene_cornell(bre_scene *s, float sigma_a, float sigma_s, float g) {
    if (!s) return;
    memset(s, 0, sizeof(*s));
    // scenes/cornell_world.pbrt: one "trianglemesh" per wall, indices [0 1 2 0 2 3]
    struct M {
        float v[4][3], kd[3];
        int emit;
    };
    const float W = 0.73f, R0 = 0.63f, R1 = 0.065f, R2 = 0.05f, G0 = 0.14f, G1 = 0.45f, G2 = 0.091f;
    const M ms[7] = {
        {{{0, 0, 0}, {0, 0, 1}, {1, 0, 1}, {1, 0, 0}}, {W, W, W}, 0},          // floor, normal +y
        {{{0, 1, 0}, {1, 1, 0}, {1, 1, 1}, {0, 1, 1}}, {W, W, W}, 0},          // ceiling, normal -y
        {{{0, 0, 1}, {0, 1, 1}, {1, 1, 1}, {1, 0, 1}}, {W, W, W}, 0},          // back wall, normal -z
        {{{0, 0, 0}, {1, 0, 0}, {1, 1, 0}, {0, 1, 0}}, {W, W, W}, 0},          // front wall (behind camera), +z
        {{{0, 0, 0}, {0, 1, 0}, {0, 1, 1}, {0, 0, 1}}, {R0, R1, R2}, 0},       // left wall (red), +x
        {{{1, 0, 0}, {1, 0, 1}, {1, 1, 1}, {1, 1, 0}}, {G0, G1, G2}, 0},       // right wall (green), -x
        {{{0.35f, 0.999f, 0.35f}, {0.65f, 0.999f, 0.35f}, {0.65f, 0.999f, 0.65f}, {0.35f, 0.999f, 0.65f}},
         {0, 0, 0}, 1},                                                         // light, normal -y
    };
    const float Le[3] = {17.f, 12.f, 4.f};
    const int idx[6] = {0, 1, 2, 0, 2, 3};
    s->n_triangles = 14;
    for (int m = 0; m < 7; ++m)
        for (int t = 0; t < 2; ++t) {
            bre_triangle &T = s->triangles[2 * m + t];
            for (int v = 0; v < 3; ++v) memcpy(T.p[v], ms[m].v[idx[3 * t + v]], 12);
            memcpy(T.kd, ms[m].kd, 12);
            T.emit = ms[m].emit;
            if (T.emit) memcpy(T.Le, Le, 12);
        }
    s->has_medium = 1;
    for (int k = 0; k < 3; ++k) {
        s->sigma_a[k] = sigma_a;
        s->sigma_s[k] = sigma_s;
    }
    s->g = g;
    const float pos[3] = {0.5f, 0.5f, 0.02f}, look[3] = {0.5f, 0.5f, 1.f}, up[3] = {0, 1, 0};
    memcpy(s->cam_pos, pos, 12);
    memcpy(s->cam_look, look, 12);
    memcpy(s->cam_up, up, 12);
    s->cam_fov_deg = 60.f;
}

void bre_scene_cornell_smoke(bre_scene *s, float sigma_a, float sigma_s, float g, int32_t n, const float *density) {
    if (!s) return;
    bre_scene_cornell(s, sigma_a, sigma_s, g);
    s->has_medium = BRE_MEDIUM_GRID;
    s->grid_n[0] = s->grid_n[1] = s->grid_n[2] = n;
    memset(s->world_to_medium, 0, sizeof(s->world_to_medium));
    for (int k = 0; k < 4; ++k) s->world_to_medium[5 * k] = 1.f;  // the grid spans the box's unit cube
    s->grid_density = density;
}

void bre_smoke_density(int32_t n, uint64_t seed, float *density) {
    if (!density || n < 1) return;
    // 3 octaves of trilinear value noise on lattices of 5, 9, 17 points per axis, values from
    // PCG32 sequence `seed` (rng.h:78-85) in lattice order
    bre::Pcg r;
    bre::pcg_seed(r, seed);
    std::vector<float> lat[3];
    int m[3];
    for (int k = 0; k < 3; ++k) {
        m[k] = (4 << k) + 1;
        lat[k].resize((size_t)m[k] * m[k] * m[k]);
        for (float &v : lat[k]) v = bre::pcg_float(r);
    }
    for (int z = 0; z < n; ++z)
        for (int y = 0; y < n; ++y)
            for (int x = 0; x < n; ++x) {
                const float p[3] = {(x + 0.5f) / n, (y + 0.5f) / n, (z + 0.5f) / n};
                float v = 0.f, amp = 0.5f;
                for (int k = 0; k < 3; ++k, amp *= 0.5f) {
                    const int L = m[k] - 1;
                    int i[3];
                    float f[3];
                    for (int a = 0; a < 3; ++a) {
                        const float q = p[a] * L;
                        i[a] = std::min((int)q, L - 1);
                        f[a] = q - (float)i[a];
                    }
                    float acc = 0.f;
                    for (int c = 0; c < 8; ++c) {
                        const int dx = c & 1, dy = (c >> 1) & 1, dz = c >> 2;
                        const float w = (dx ? f[0] : 1 - f[0]) * (dy ? f[1] : 1 - f[1]) * (dz ? f[2] : 1 - f[2]);
                        acc += w * lat[k][((size_t)(i[2] + dz) * m[k] + (i[1] + dy)) * m[k] + (i[0] + dx)];
                    }
                    v += amp * acc;
                }
                const float dx = p[0] - 0.5f, dy = p[1] - 0.45f, dz = p[2] - 0.55f;
                const float rr = std::sqrt(dx * dx + dy * dy + dz * dz);
                const float shape = std::min(1.f, std::max(0.f, (0.45f - rr) / 0.2f));
                density[((size_t)z * n + y) * n + x] = std::max(0.f, 2.f * v - 0.4f) * shape;
            }
}

bre_status bre_gather_device(bre_ctx *c, int64_t nseg, const float *o, const float *p, const float *d,
                             const float *tmax, const int32_t *pixel, float R, int64_t npix, float *accum,
                             float *seg_rgb, int32_t *seg_counts) {
    if (!c) return BRE_ERR_INVALID_ARG;
    bre_status st = set_device(c);
    if (st != BRE_OK) return st;
    return gather_segments(c, nseg, o, p, d, tmax, pixel, R, npix, accum, seg_rgb, seg_counts);
}

bre_status bre_gather(bre_ctx *c, int64_t nseg, const float *o, const float *p, const float *d, const float *tmax,
                      const int32_t *pixel, float R, int64_t npix, float *accum, float *seg_rgb,
                      int32_t *seg_counts) {
    if (!c) return BRE_ERR_INVALID_ARG;
    if (nseg < 0 || npix < 0) return fail(c, BRE_ERR_INVALID_ARG, "bre_gather: negative size");
    if (c->film_classes > 1 && accum)
        return fail(c, BRE_ERR_STATE, "bre_gather: BRE_OPT_FILM_CLASSES is for caller device films (bre_gather_device)");
    if (nseg > 0 && (!o || !p || !d || !tmax))
        return fail(c, BRE_ERR_INVALID_ARG, "bre_gather: null segment array");
    if (accum && !pixel) return fail(c, BRE_ERR_INVALID_ARG, "bre_gather: accum_rgb given without seg_pixel");
    if (accum && pixel) {
        for (int64_t s = 0; s < nseg; ++s)
            if (pixel[s] < 0 || pixel[s] >= npix)
                return fail(c, BRE_ERR_INVALID_ARG, "bre_gather: seg_pixel[%lld]=%d out of [0,%lld)", (long long)s,
                            pixel[s], (long long)npix);
    }
    bre_status st = set_device(c);
    if (st != BRE_OK) return st;
    const size_t S = (size_t)nseg, P = (size_t)npix;
    if (nseg == 0) return BRE_OK;
    HIPCHK(c, c->g_o.ensure(S * 3 * sizeof(float)));
    HIPCHK(c, c->g_p.ensure(S * 3 * sizeof(float)));
    HIPCHK(c, c->g_d.ensure(S * 3 * sizeof(float)));
    HIPCHK(c, c->g_tmax.ensure(S * sizeof(float)));
    HIPCHK(c, hipMemcpyAsync(c->g_o.ptr, o, S * 3 * sizeof(float), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->g_p.ptr, p, S * 3 * sizeof(float), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->g_d.ptr, d, S * 3 * sizeof(float), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->g_tmax.ptr, tmax, S * sizeof(float), hipMemcpyHostToDevice, c->stream));
    int32_t *dpix = nullptr;
    float *daccum = nullptr, *dseg = nullptr;
    int32_t *dcnt = nullptr;
    if (pixel) {
        HIPCHK(c, c->g_pix.ensure(S * sizeof(int32_t)));
        HIPCHK(c, hipMemcpyAsync(c->g_pix.ptr, pixel, S * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
        dpix = c->g_pix.as<int32_t>();
    }
    if (accum && npix > 0) {
        HIPCHK(c, c->g_accum.ensure(P * 3 * sizeof(float)));
        HIPCHK(c, hipMemcpyAsync(c->g_accum.ptr, accum, P * 3 * sizeof(float), hipMemcpyHostToDevice, c->stream));
        daccum = c->g_accum.as<float>();
    }
    if (seg_rgb) {
        HIPCHK(c, c->g_seg_rgb.ensure(S * 3 * sizeof(float)));
        dseg = c->g_seg_rgb.as<float>();
    }
    if (seg_counts) {
        HIPCHK(c, c->g_counts.ensure(S * 2 * sizeof(int32_t)));
        dcnt = c->g_counts.as<int32_t>();
    }
    st = gather_segments(c, nseg, c->g_o.as<float>(), c->g_p.as<float>(), c->g_d.as<float>(), c->g_tmax.as<float>(),
                         dpix, R, npix, daccum, dseg, dcnt);
    if (st != BRE_OK) return st;
    if (daccum) HIPCHK(c, hipMemcpyAsync(accum, daccum, P * 3 * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    if (dseg) HIPCHK(c, hipMemcpyAsync(seg_rgb, dseg, S * 3 * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    if (dcnt) HIPCHK(c, hipMemcpyAsync(seg_counts, dcnt, S * 2 * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    return check_flags(c);
}

}  // extern "C"

// ---- multi-GPU: one host thread per context ----
namespace {
struct ShardSave {
    int mode, count, rank, block;
};
// Run fn(i) for every context on its own thread (fn(0) on the caller's); the first failing
// context's status and message (prefixed with its index) end up in ctxs[0].
template <typename Fn>
bre_status for_each_ctx(bre_ctx *const *ctxs, int n, Fn fn) {
    std::vector<bre_status> st((size_t)n, BRE_OK);
    std::vector<std::thread> th;
    th.reserve((size_t)n);
    for (int i = 1; i < n; ++i) th.emplace_back([&, i] { st[(size_t)i] = fn(i); });
    st[0] = fn(0);
    for (auto &t : th) t.join();
    for (int i = 0; i < n; ++i) {
        if (st[(size_t)i] == BRE_OK) continue;
        const std::string msg = "context " + std::to_string(i) + ": " + ctxs[i]->err;
        ctxs[0]->err = msg;
        return st[(size_t)i];
    }
    return BRE_OK;
}
bre_status check_ctxs(bre_ctx *const *ctxs, int n) {
    if (!ctxs || n < 1) return BRE_ERR_INVALID_ARG;
    for (int i = 0; i < n; ++i) {
        if (!ctxs[i]) return BRE_ERR_INVALID_ARG;
        for (int j = 0; j < i; ++j)
            if (ctxs[j] == ctxs[i]) return fail(ctxs[0], BRE_ERR_INVALID_ARG, "bre_*_sharded: context %d repeated", i);
    }
    return BRE_OK;
}
}  // namespace

extern "C" {

bre_status bre_set_beams_sharded(bre_ctx *const *ctxs, int n_ctx, int64_t n, const float *start, const float *end,
                                 const float *radius, const float *power) {
    bre_status st = check_ctxs(ctxs, n_ctx);
    if (st != BRE_OK) return st;
    return for_each_ctx(ctxs, n_ctx, [&](int i) { return bre_set_beams(ctxs[i], n, start, end, radius, power); });
}

bre_status bre_gather_sharded(bre_ctx *const *ctxs, int n_ctx, int64_t nseg, const float *o, const float *p,
                              const float *d, const float *tmax, const int32_t *pixel, float R, int64_t npix,
                              float *accum, float *seg_rgb, int32_t *seg_counts) {
    bre_status st = check_ctxs(ctxs, n_ctx);
    if (st != BRE_OK) return st;
    if (nseg < 0 || npix < 0) return fail(ctxs[0], BRE_ERR_INVALID_ARG, "bre_gather_sharded: negative size");
    for (int i = 0; i < n_ctx; ++i)
        if (ctxs[i]->film_classes > 1)
            return fail(ctxs[0], BRE_ERR_STATE, "bre_gather_sharded: BRE_OPT_FILM_CLASSES is for caller device films");
    const size_t F = accum && npix > 0 ? (size_t)npix * 3 : 0, S = (size_t)nseg;
    // per context: its partial film and per-segment outputs (only its own packets' entries are
    // nonzero); the contexts' shard options are set for the call and restored afterwards
    std::vector<std::vector<float>> film((size_t)n_ctx), rgb((size_t)n_ctx);
    std::vector<std::vector<int32_t>> cnt((size_t)n_ctx);
    std::vector<ShardSave> saved((size_t)n_ctx);
    for (int i = 0; i < n_ctx; ++i) {
        bre_ctx *c = ctxs[i];
        saved[(size_t)i] = ShardSave{c->shard_mode, c->shard_count, c->shard_rank, c->shard_block};
        c->shard_mode = 1;
        c->shard_count = n_ctx;
        c->shard_rank = i;
        c->shard_block = 1;
    }
    st = for_each_ctx(ctxs, n_ctx, [&](int i) {
        const size_t k = (size_t)i;
        film[k].assign(F, 0.f);
        if (seg_rgb) rgb[k].assign(S * 3, 0.f);
        if (seg_counts) cnt[k].assign(S * 2, 0);
        return bre_gather(ctxs[i], nseg, o, p, d, tmax, pixel, R, npix, F ? film[k].data() : nullptr,
                          seg_rgb ? rgb[k].data() : nullptr, seg_counts ? cnt[k].data() : nullptr);
    });
    for (int i = 0; i < n_ctx; ++i) {
        bre_ctx *c = ctxs[i];
        const ShardSave &v = saved[(size_t)i];
        c->shard_mode = v.mode;
        c->shard_count = v.count;
        c->shard_rank = v.rank;
        c->shard_block = v.block;
    }
    if (st != BRE_OK) return st;
    // the films in context order (deterministic), then into the caller's Ld
    for (size_t j = 0; j < F; ++j) {
        float v = film[0][j];
        for (int i = 1; i < n_ctx; ++i) v += film[(size_t)i][j];
        accum[j] += v;
    }
    if (seg_rgb)
        for (size_t j = 0; j < S * 3; ++j) {
            float v = rgb[0][j];
            for (int i = 1; i < n_ctx; ++i) v += rgb[(size_t)i][j];  // one nonzero term per entry
            seg_rgb[j] = v;
        }
    if (seg_counts)
        for (size_t j = 0; j < S * 2; ++j) {
            int32_t v = cnt[0][j];
            for (int i = 1; i < n_ctx; ++i) v += cnt[(size_t)i][j];
            seg_counts[j] = v;
        }
    return BRE_OK;
}

int64_t bre_shard_segments(int64_t n_segments, int32_t rank, int32_t count, int32_t chunk) {
    if (n_segments <= 0) return 0;
    if (count <= 1) return n_segments;
    if (rank < 0 || rank >= count || chunk < 1) return 0;
    const int64_t npk = (n_segments + 63) / 64, K = chunk;
    const int64_t nch = (npk + K - 1) / K;                              // chunks of K packets
    const int64_t q = rank < nch ? (nch - 1 - rank) / count + 1 : 0;    // chunks c = rank (mod count)
    const bool last = (nch - 1) % count == rank;                        // owns the only partial chunk
    const int64_t packets = q * K - (last ? nch * K - npk : 0);
    return packets * 64 - (last ? npk * 64 - n_segments : 0);
}

bre_status bre_device_check(bre_ctx *c, int32_t kind, int64_t n, const float *x, int32_t n_aux, const float *aux,
                            float *y) {
    if (!c) return BRE_ERR_INVALID_ARG;
    if (kind < 0 || kind > 9) return fail(c, BRE_ERR_INVALID_ARG, "bre_device_check: kind %d not in [0, 9]", kind);
    if (n < 0 || (n > 0 && (!x || !y))) return fail(c, BRE_ERR_INVALID_ARG, "bre_device_check: bad arrays");
    if (kind >= 6 && kind <= 8) {
        // the pass chain's one-wave primitives (bre_slot.hip) on caller data
        bre_status st = set_device(c);
        if (st != BRE_OK) return st;
        if (n == 0) return BRE_OK;
        if (kind == 7) {  // exclusive scan of n int32 words; y: n + 1 int64 (the total last)
            HIPCHK(c, c->chk_x.ensure((size_t)n * 4));
            HIPCHK(c, c->chk_y.ensure((size_t)(n + 1) * 8));
            HIPCHK(c, c->chk_aux.ensure(slot_scan_temp_bytes(n)));
            HIPCHK(c, hipMemcpyAsync(c->chk_x.ptr, x, (size_t)n * 4, hipMemcpyHostToDevice, c->stream));
            HIPCHK(c, slot_exclusive_scan(c->chk_x.as<int32_t>(), c->chk_y.as<int64_t>(), n, c->chk_y.as<int64_t>() + n,
                                          c->chk_aux.ptr, c->stream));
            HIPCHK(c, hipMemcpyAsync(y, c->chk_y.ptr, (size_t)(n + 1) * 8, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
            return BRE_OK;
        }
        // kind 6 / 8: stable sort of m = n / 2 64-bit (n 32-bit) keys by bits [aux[0], aux[1]), values = the
        // input positions; y: the sorted keys, then the values
        if (n_aux < 2 || !aux) return fail(c, BRE_ERR_INVALID_ARG, "bre_device_check: kinds 6 / 8 need aux[0..1] bits");
        const int kb = kind == 6 ? 8 : 4;
        if ((n * 4) % kb) return fail(c, BRE_ERR_INVALID_ARG, "bre_device_check: kind 6 needs an even word count");
        const int64_t m = n * 4 / kb;
        const size_t tb = slot_sort_temp_bytes(m, kb);
        HIPCHK(c, c->chk_x.ensure((size_t)m * (kb + 4) * 2 + tb + 512));
        char *base = static_cast<char *>(c->chk_x.ptr);
        char *k0 = base, *k1 = k0 + (size_t)m * kb, *v0 = k1 + (size_t)m * kb, *v1 = v0 + (size_t)m * 4;
        void *tmp = v1 + ((size_t)m * 4 + 256) / 256 * 256;
        std::vector<int32_t> idx((size_t)m);
        for (int64_t i = 0; i < m; ++i) idx[(size_t)i] = (int32_t)i;
        HIPCHK(c, hipMemcpyAsync(k0, x, (size_t)m * kb, hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipMemcpyAsync(v0, idx.data(), (size_t)m * 4, hipMemcpyHostToDevice, c->stream));
        const int b0 = (int)aux[0], b1 = (int)aux[1];
        if (kb == 8)
            HIPCHK(c, slot_sort_pairs(tmp, reinterpret_cast<unsigned long long *>(k0), reinterpret_cast<unsigned long long *>(k1),
                                      reinterpret_cast<int32_t *>(v0), reinterpret_cast<int32_t *>(v1), m, b0, b1, c->stream));
        else
            HIPCHK(c, slot_sort_pairs(tmp, reinterpret_cast<unsigned int *>(k0), reinterpret_cast<unsigned int *>(k1),
                                      reinterpret_cast<int32_t *>(v0), reinterpret_cast<int32_t *>(v1), m, b0, b1, c->stream));
        HIPCHK(c, hipMemcpyAsync(y, k1, (size_t)m * kb, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipMemcpyAsync(reinterpret_cast<char *>(y) + (size_t)m * kb, v1, (size_t)m * 4, hipMemcpyDeviceToHost,
                                 c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        return BRE_OK;
    }
    if (kind == 5) {
        // the tile kernel's work roots (k_roots) of a caller tree: x = n / 16 Node records as words
        if (n_aux < 1 || !aux) return fail(c, BRE_ERR_INVALID_ARG, "bre_device_check: kind 5 needs aux[0] = S");
        const int S = (int)aux[0];
        if (n < 16 || n % 16 || S < 1 || S > kMaxSplit || (S & (S - 1)))
            return fail(c, BRE_ERR_INVALID_ARG, "bre_device_check: kind 5 needs whole Node records and S a power of two <= %d",
                        kMaxSplit);
        bre_status st = set_device(c);
        if (st != BRE_OK) return st;
        HIPCHK(c, c->chk_x.ensure((size_t)n * 4));
        HIPCHK(c, c->chk_y.ensure((size_t)(S + 1) * 4));
        HIPCHK(c, hipMemcpyAsync(c->chk_x.ptr, x, (size_t)n * 4, hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, c->roots_tmp.ensure(roots_scratch_bytes()));
        HIPCHK(c, launch_roots(c->chk_x.as<Node>(), S, c->chk_y.as<int32_t>(), c->roots_tmp.ptr, c->stream));
        HIPCHK(c, hipMemcpyAsync(y, c->chk_y.ptr, (size_t)(S + 1) * 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        return BRE_OK;
    }
    const bool need_aux = kind == 3 || kind == 4;
    if (need_aux && (n_aux < 1 || !aux)) return fail(c, BRE_ERR_INVALID_ARG, "bre_device_check: kind %d needs aux", kind);
    if (n == 0) return BRE_OK;
    bre_status st = set_device(c);
    if (st != BRE_OK) return st;
    const int64_t outs = kind == 9 ? 4 * n : (kind == 2 || kind == 4) ? 2 * n : n;
    HIPCHK(c, c->chk_x.ensure((size_t)n * 4));
    HIPCHK(c, c->chk_y.ensure((size_t)outs * 4));
    HIPCHK(c, c->chk_aux.ensure(need_aux ? (size_t)n_aux * 4 : 4));
    HIPCHK(c, hipMemcpyAsync(c->chk_x.ptr, x, (size_t)n * 4, hipMemcpyHostToDevice, c->stream));
    if (need_aux)
        HIPCHK(c, hipMemcpyAsync(c->chk_aux.ptr, aux, (size_t)n_aux * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, launch_device_check(kind, n, c->chk_x.as<float>(), need_aux ? n_aux : 0, c->chk_aux.as<float>(),
                                  c->chk_y.as<float>(), c->stream));
    HIPCHK(c, hipMemcpyAsync(y, c->chk_y.ptr, (size_t)outs * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return BRE_OK;
}

float bre_beam_radius_at(float initial_radius, float alpha, int iteration) {
    float r = initial_radius;
    for (int i = 0; i < iteration; ++i) r = r * (float(i + alpha) / float(i + 1));
    return r;
}

bre_status bre_resolve_image(int64_t npix, const float *ld, int iteration, float *out) {
    if (npix < 0 || (npix > 0 && (!ld || !out)) || iteration < 0) return BRE_ERR_INVALID_ARG;
    // Spectrum L = pixel.Ld / (iter + 1): operator/(Float) divides each channel (spectrum.h:180-186)
    const float div = (float)(iteration + 1);
    for (int64_t i = 0; i < 3 * npix; ++i) out[i] = ld[i] / div;
    return BRE_OK;
}

}  // extern "C"
