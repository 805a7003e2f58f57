// bre_device.h — device data layout and kernel launchers shared by the build and gather units.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bre {

// One beam in BVH (sorted) order: 64 B, one cache line.  Everything the per-pair test needs.
// When every valid beam of the set has the same radius (BeamSet::uniform: the integrator's own beams
// always do, photonbeam.cpp:292 stores the pass radius in each), the radius is the set's and the last
// three words hold the beam's scaled power (the float4 power array's x, y, z), so a contributing pair
// reads one record instead of a record and a power line.
struct alignas(16) BeamRec {
    float lo[3], hi[3];  // reference test box: WorldBound, or the union over beams with an
                         // identical centroid (those share one SAH leaf in the reference)
    float b0[3];         // beam start
    float bu[3];         // (end - start) * (1/|end - start|)
    float mag_b;         // |end - start|
    float radius;        // beam radius (PhotonBeam::radius); uniform sets: power.x
    float pad[2];        // uniform sets: power.y, power.z
};
// How a gather reads a BeamRec's radius and power (the build's finding, passed by value).
struct BeamSet {
    int uniform = 0;      // 1: every valid beam has radius `radius`, power in the record's last words
    float radius = 0.f;
};
__device__ __forceinline__ float beam_radius(const BeamSet &u, float rec_radius) {
    return u.uniform ? u.radius : rec_radius;
}
static_assert(sizeof(BeamRec) == 64, "BeamRec must be one 64-B line");

// Binary BVH interior node, 64 B: both children's boxes live in the parent so one line per
// visit tests two children.  child >= 0: interior node index; child < 0: leaf cluster ~child;
// kEmptyChild: no child (box is empty).
struct alignas(16) Node {
    float lo[2][3];
    float hi[2][3];
    int32_t child[2];
    int32_t parent;
    int32_t nleaf;  // leaf tiles below this node (k_karras: its key range; the work-root split sizes by it)
};
static_assert(sizeof(Node) == 64, "Node must be one 64-B line");

constexpr int32_t kEmptyChild = INT32_MIN;

// The tile kernel's 4-wide view of the binary tree (k_collapse4): record i holds the boxes and
// indices of binary node i's grandchildren, in left-to-right order (a leaf child stands for itself,
// empty slots are kEmptyChild), so one node visit tests two levels of the tree.  Boxes are SoA
// (lo[axis][slot]) so a visit reads the record with two 64-B scalar loads.
struct alignas(16) Node4 {
    float lo[3][4], hi[3][4];
    int32_t child[4];
    int32_t pad[4];
};
static_assert(sizeof(Node4) == 128, "Node4 must be two 64-B lines");
constexpr int kStackDepth = 128;     // wave-uniform traversal stack (entries per wave)
constexpr int kThreadStackDepth = 64;  // per-thread stack of the thread-per-segment kernel
constexpr int kMaxSplit = 1024;         // max work roots (subtrees) per gather

// DevCounters::flags bits.  The host reads the word at every synchronising call and turns a set bit
// into an error (bre_api.hip: check_flags), whatever the counters option.
constexpr unsigned int kFlagStack = 1u;  // a traversal stack overflowed: contributions were dropped
constexpr unsigned int kFlagPixel = 2u;  // a seg_pixel index outside [0, npix): the segment was skipped

// Error / counter block in device memory (the counters are zeroed per gather; `flags` is sticky
// until the host has read it).
struct DevCounters {
    unsigned long long candidates;
    unsigned long long contributions;
    unsigned long long node_visits;
    unsigned long long leaf_visits;        // leaf tiles visited (per wave)
    unsigned long long beam_evals;         // beam records staged (per wave)
    unsigned long long ccp_wave_evals;     // exact-stage batches of <= 64 pairs (per wave)
    unsigned long long prefilter_rejects;  // lane-level candidate rejects by the line-distance prefilters
    unsigned long long useful_beam_evals;  // beams kept by the packet bundle test
    unsigned long long queued_pairs;       // tile kernel, counters: (lane, beam) pairs queued for the exact stage
    unsigned int max_stack;
    unsigned int flags;  // kFlag* bits (sticky)
};

struct BuildBuffers {
    // inputs (device)
    const float *start, *end, *radius, *power;
    int64_t n;
    int sqrt_mode;
    int leaf_size;
    int beam_key = 2;  // tree order: 2 Hilbert of (start, end) (default), 1 Morton of (start, end), 0 Morton of the centroid
    // scratch
    float *box;        // 6n (input order)
    float *cent;       // 3n (input order)
    unsigned int *cbounds;  // 12 ordered uints: min/max of valid centroids, then of their end points
    float *gbox;            // 6n (input order): equal-centroid group boxes (tree key 1)
    unsigned int *nvalid;   // 3: valid beams, then the ordered min and max of their radii
    int uniform_radius = 0; // k_pack: the set's BeamSet::uniform (read back after k_prep)
    int slot = 1;           // sorts and fills by the one-wave primitives (bre_slot.hip), 0: rocPRIM / hipMemset
    int key_lo = 0;         // the tree-order sort skips the key's bits below key_lo (internal option 121)
    unsigned long long *keys, *keys_alt;
    int32_t *vals, *vals_alt;
    void *sort_tmp;
    size_t sort_tmp_bytes;
    int32_t *leaf_parent;  // nleaf
    unsigned int *visit;   // nnodes counters
    // outputs
    BeamRec *recs;      // nvalid
    float4 *pow;        // nvalid, powerEnd * 1e-5f
    Node *nodes;        // max(nleaf-1, 1)
    // capacities (elements) of the hierarchy's output / scratch buffers, checked by launch_hierarchy
    uint64_t nodes_cap = 0, leaf_parent_cap = 0, visit_cap = 0;
};

// One capsule chunk of a beam LINE (kernel 5, bre_chunk.hip): 64 B, same leading lo/hi as
// BeamRec so the LBVH kernels (k_morton / k_karras / k_refit) build over chunks unchanged.
struct alignas(16) ChunkRec {
    float lo[3], hi[3];  // conservative box: the chunk's line piece expanded by E = (R + r)(1+1e-3)+margin
    float b0[3];         // parent beam start   (ComputeClosestPoints inputs, exactly the parent's)
    float bu[3];         // parent unit direction
    float mag_b;         // parent |end - start|
    float radius;        // parent radius
    float s_lo, s_hi;    // ownership: the pair belongs to this chunk iff s_lo <= s < s_hi, s = the
                         // line parameter of ComputeClosestPoints' beam point
};
static_assert(sizeof(ChunkRec) == 64, "ChunkRec must be one 64-B line");

// build kernels (bre_build.hip)
hipError_t launch_prep(const BuildBuffers &b, hipStream_t s);
hipError_t launch_morton(const BuildBuffers &b, hipStream_t s);
size_t sort_temp_bytes(int64_t n);
// tree keys 1 / 2: a hash of the centroid for the equal-centroid groups (sorted over 32 bits)
hipError_t launch_cent_hash(const BuildBuffers &b, hipStream_t s);
hipError_t launch_sort(const BuildBuffers &b, hipStream_t s, int end_bit = 64, int begin_bit = 0);
hipError_t launch_pack(const BuildBuffers &b, int64_t nvalid, hipStream_t s);
// tree key 1, after the centroid sort: group boxes (k_group), then the (start, end) keys into keys/vals
hipError_t launch_tree_key(const BuildBuffers &b, int64_t nvalid, hipStream_t s);
hipError_t launch_hierarchy(const BuildBuffers &b, int64_t nvalid, hipStream_t s);

// One gathered segment as the tile kernel's exact stage reads it (k_seg_prep): 64 B as four 16-B
// planes.  In HBM the records are stored PLANE-MAJOR PER PACKET of 64 segments (seg_plane): plane k of
// the packet's 64 segments is one contiguous 1 KB run, so an exact-stage load of plane k for 64
// arbitrary lanes of the packet touches at most 1 KB (16 lines) instead of 64 separate lines.
struct alignas(16) SegRec {
    float o[3], tmax;   // ray.o, ray.tMax
    float p[3], mag_a;  // isect.p, |p - o|, negated (sign bit set) when some 1 / d_i is infinite
    float au[3];        // (p - o) * (1 / |p - o|)
    int32_t has_inf;    // some 1 / d_i is infinite (axis-parallel ray)
    float invs[3];      // 1 / d with infinities replaced by +-FLT_MAX
    float inv_mag_a;    // RN(1 / |p - o|) (0 for a zero-length segment): the tile kernel's exact stage
                        // reads planes 0, 1 and 3 and recomputes au = (p - o) * inv_mag_a
};
static_assert(sizeof(SegRec) == 64, "SegRec must be one 64-B line");
// plane k (0..3) of segment s in the packet-plane layout (buffers hold ceil(nseg / 64) * 64 records)
__device__ __forceinline__ const float4 *seg_plane(const SegRec *base, int64_t s, int k) {
    return reinterpret_cast<const float4 *>(base) + ((s >> 6) << 8) + (k << 6) + (s & 63);
}

// Per leaf tile of the tile kernel's tree, per gather (k_tile_axis): an axis line p + s d (|d| = 1)
// such that every beam LINE of the tile, clipped to the box of the gather's segments grown by
// (R + rmax) and a margin, lies within rho of it -- stored as the scan's separable record of a
// pseudo-beam: d, m = d x p and thr = rho + the beam-side prefilter margin Ab' (maxd = R + rmax);
// live < 0: no beam of the tile can contribute at all.
struct alignas(16) TileAxis {
    float d[3], thr;
    float m[3], grow;  // grow: the region's growth maxd_max + margins; < 0: no beam of the tile can contribute
};

struct GatherArgs {
    int64_t nseg;
    const float *o, *p, *d, *tmax;
    const int32_t *pixel;
    float R;
    int64_t npix;
    float *accum;          // may be null
    float *seg_rgb;        // may be null
    int32_t *seg_counts;   // may be null
    const int32_t *seg_index;  // may be null: seg_rgb / seg_counts entry of gathered segment s is seg_index[s]
    const BeamRec *recs;
    const float4 *pow;
    BeamSet bset;
    const Node *nodes;
    const Node4 *nodes4 = nullptr;  // tile kernel: the 4-wide view of `nodes` (null: binary traversal)
    int64_t nvalid;
    int leaf_size;
    DevCounters *ctr;
    // tile kernel: subtree split
    const int32_t *roots;  // [split] work roots + [split] = count
    int split;             // S, power of two <= kMaxSplit
    float *partial;        // [split][nseg][3]
    int32_t *pcnt;         // [split][nseg][2] per-subtree counts (counters / contribution counting)
    SegRec *segrec;        // [nseg] tile kernel: per-segment records (written by k_seg_prep)
    bool prefilter;
    int occupancy;         // tile kernel register budget: min waves per SIMD (1, 6, 7 or 8)
    int stack_cap;         // traversal stack entries to use (0 = all); tests force an overflow
    int block_map;         // tile kernel block -> (packet, subtree) mapping (k_gather_tile)
    int tscan;             // tile kernel: transposed scan when on-lanes * 8 < kept beams * tscan (0: off)
    int margin;            // tile kernel prefilter margins: 1 = the tight bound (default), 0 = round 2's
    TileAxis *tileax;      // tile kernel: per-tile axis bounds (ntiles), null = no tile axis reject
    unsigned int *segbox;  // tile kernel: 6 ordered uints of scratch (the launch's segment box)
    hipEvent_t wait_ev = nullptr;  // tile kernel: the stream waits for it right before the launch (null: no wait)
    hipEvent_t done_ev = nullptr;  // tile kernel: recorded right after the launch (null: none)
    hipEvent_t user_start = nullptr, user_end = nullptr;  // caller's timing events (bre_set_gather_events)
};

// capsule-chunk index (bre_chunk.hip)
struct ChunkBuild {
    const BeamRec *parents;   // sorted parent beam records (reference group boxes)
    BeamSet bset;
    int64_t nparents;
    const float *seg_o, *seg_p;  // the gather's segments (clip box)
    int64_t nseg;
    float R;
    float len_factor;         // chunk length = len_factor * E
    unsigned int *seg_bounds;  // 6 ordered uints (scratch)
    unsigned int *cbounds;     // 6 ordered uints (scratch)
    int32_t *counts;           // nparents + 1
    int64_t *offsets;          // nparents + 1
    float *range;              // 2 * nparents
    void *scan_tmp;
    size_t scan_tmp_bytes;
};
size_t chunk_scan_temp_bytes(int64_t n);
// pass 1: clip every parent's line to the segments' box, count its chunks; *total after the scan
hipError_t launch_chunk_count(const ChunkBuild &c, hipStream_t s);
// pass 2: emit chunk boxes / centroids (input order) + temp fields
hipError_t launch_chunk_emit(const ChunkBuild &c, float *box, float *cent, float *s_lo, float *s_hi,
                             int32_t *parent, hipStream_t s);
// pass 3 (after morton + sort): sorted ChunkRecs + their parent indices
hipError_t launch_chunk_pack(const ChunkBuild &c, int64_t nchunks, const int32_t *order, const float *box,
                             const float *s_lo, const float *s_hi, const int32_t *parent, ChunkRec *out,
                             int32_t *out_parent, hipStream_t s);
struct ChunkGatherArgs {
    int64_t nseg;
    const float *o, *p, *d, *tmax;
    const int32_t *pixel;
    float R;
    int64_t npix;
    float *accum, *seg_rgb;
    int32_t *seg_counts;
    const ChunkRec *chunks;
    const int32_t *chunk_parent;
    const BeamRec *parents;
    const float4 *pow;
    const Node *nodes;
    int64_t nchunks;
    int leaf_size;
    bool prefilter;
    DevCounters *ctr;
};
hipError_t launch_gather_chunk(const ChunkGatherArgs &a, bool counters, hipStream_t s);

// coherence sort of a gather's segments (bre_sort.hip): 5-D Morton of (origin, direction)
struct SegSort {
    int64_t n;
    const float *o, *p, *d, *t;
    const int32_t *pix;
    unsigned int *bounds;  // 6
    unsigned long long *keys, *keys_alt;
    int32_t *vals, *vals_alt;
    void *tmp;
    size_t tmp_bytes;
    float *o2, *p2, *d2, *t2;  // sorted copies
    int32_t *pix2;
    int key_mode;  // 0: Morton of (origin, octahedral direction); 1: Morton of (origin, end point);
                   // 2 / 3: the segment's line (dominant-axis class + slopes + plane crossing [+ midpoint]);
                   // 4: Hilbert order of (origin, end point) (the default, bre_math.h hilbert_key)
    int slot = 1;  // the sort by the one-wave radix sort (bre_slot.hip), 0: rocPRIM
    int key_lo = 0;  // the sort skips the key's bits below key_lo (coarse keys, internal option 121)
};
size_t seg_sort_temp_bytes(int64_t n);
// deterministic per-pixel accumulation of per-segment sums (bre_sort.hip): stable sort of the
// segments by pixel, then one thread per pixel adds its segments in the caller's order
struct PixelCompose {
    int64_t n;
    const int32_t *pix;      // [n] pixel of each segment
    const float *seg_rgb;    // [3n] per-segment sums
    int64_t npix;
    float *accum;            // [3 npix] += per pixel; with classes: [classes][3 npix]
    const uint8_t *cls;      // [n] film class of each segment (nullptr: one film)
    int classes;             // 1 or BRE_FILM_CLASSES
    unsigned int *keys, *keys_alt;
    int32_t *vals, *vals_alt;
    void *tmp;
    size_t tmp_bytes;
    unsigned int *flags;     // DevCounters::flags
    unsigned int bad_pixel_flag;
    int slot = 1;            // the sort by the one-wave radix sort (bre_slot.hip), 0: rocPRIM
};
size_t pixel_sort_temp_bytes(int64_t n);
hipError_t launch_pixel_compose(const PixelCompose &c, hipStream_t st);
// film class of each caller-order segment: chunk (sorted position / 64 / block) mod classes; perm[i] =
// the caller index of sorted segment i (nullptr: unsorted, the caller's order)
hipError_t launch_seg_classes(int64_t n, int block, int classes, const int32_t *perm, uint8_t *cls, hipStream_t st);
// dst[i] += src[i] for i < m, then src[i] = 0 if clear (one-wave workgroups)
hipError_t launch_film_add(int64_t m, float *src, float *dst, int clear, hipStream_t st);
// out[i] = sum over the classes of in[c][i] in class order, i < m
hipError_t launch_resolve_classes(int64_t m, int classes, const float *in, float *out, hipStream_t st);

hipError_t launch_sort_segments(const SegSort &s, hipStream_t st);
hipError_t launch_packet_pick(int64_t n, int64_t m, int rank, int count, int chunk, const float *o, const float *p,
                              const float *d, const float *t, const int32_t *pix, const int32_t *index, float *o2,
                              float *p2, float *d2, float *t2, int32_t *pix2, int32_t *index2, hipStream_t st);

// device self-check of the shared scalar primitives (bre_check.hip, bre_device_check)
hipError_t launch_device_check(int kind, int64_t n, const float *x, int n_aux, const float *aux, float *y,
                               hipStream_t s);

// one-wave pass primitives (bre_slot.hip): every kernel in 64-thread workgroups with <= 1 KB of LDS, so
// that a concurrent gather's retiring one-wave slots take them (the pipelined pass chain)
hipError_t slot_fill(void *p, int64_t nwords, unsigned int value, hipStream_t s);
size_t slot_scan_temp_bytes(int64_t n);
// out[i] = in[0] + ... + in[i-1] for i < n; *total (may be null) = the whole sum
hipError_t slot_exclusive_scan(const int32_t *in, int64_t *out, int64_t n, int64_t *total, void *tmp, hipStream_t s);
size_t slot_sort_temp_bytes(int64_t n, int key_bytes);
// stable LSD radix sort of (k0, v0) by key bits [begin_bit, end_bit) into (k1, v1); (k0, v0) unchanged
hipError_t slot_sort_pairs(void *tmp, const unsigned long long *k0, unsigned long long *k1, const int32_t *v0,
                           int32_t *v1, int64_t n, int begin_bit, int end_bit, hipStream_t s);
hipError_t slot_sort_pairs(void *tmp, const unsigned int *k0, unsigned int *k1, const int32_t *v0, int32_t *v1,
                           int64_t n, int begin_bit, int end_bit, hipStream_t s);

// gather kernels (bre_gather.hip)
size_t roots_scratch_bytes();
hipError_t launch_roots(const Node *nodes, int S, int32_t *roots, void *scratch, hipStream_t s);
hipError_t launch_collapse4(const Node *nodes, int64_t nnodes, Node4 *out, hipStream_t s);
hipError_t launch_roots_shard(const int32_t *roots, int S, int rank, int count, int S2, int32_t *out,
                              hipStream_t s);
hipError_t launch_gather(const GatherArgs &a, int kernel, bool counters, hipStream_t s);
hipError_t launch_zero_outputs(const GatherArgs &a, hipStream_t s);

}  // namespace bre
