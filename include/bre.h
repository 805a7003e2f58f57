/*
 * bre.h — C ABI of the MI355X beam-radiance-estimate (photon-beam gather) library, libbre.so.
 *
 * Drop-in boundary for the hot path of bwiberg/beam-radiance-estimate-pbrt:
 *
 *   reference (pbrt-v3 fork)                                   this ABI
 *   ---------------------------------------------------------  ---------------------------------
 *   PhotonBeamBVH photonBeamBVH(std::move(photonBeams));       bre_set_beams / bre_set_beams_device
 *     src/integrators/photonbeam.cpp:438,                        (copy + GPU build; the beam set and
 *     ctor src/core/photonbeambvh.cpp:204-248                    BVH live on the device until replaced)
 *   photonBeamBVH.Intersect(ray) + ComputeClosestPoints +      bre_gather / bre_gather_device
 *     `pixel.Ld += 1e-5 * powerEnd * sqrt(1 - r*r)`             (all camera segments of one iteration
 *     src/integrators/photonbeam.cpp:494-508,                    in one call; += into per-pixel RGB)
 *     src/core/photonbeambvh.cpp:685-723
 *   currentBeamRadius (photonbeam.cpp:354-356, 562)            argument `beam_radius_cur` (R_cur)
 *   PhotonBeam{start,end,radius,powerStart,powerEnd}           SoA/xyz float arrays below
 *     src/core/photonbeambvh.h:48-73                             (powerStart is always 0 in the
 *                                                                reference, photonbeam.cpp:266,292,
 *                                                                and unused by the gather)
 *
 * A "segment" is one camera-ray segment of the reference's camera pass: ray.o, ray.d and
 * ray.tMax after Scene::Intersect (primitive.cpp:101 sets tMax to the hit) and isect.p.
 * All four are needed: the candidate test uses (o, d, tMax) (Bounds3::IntersectP,
 * geometry.h:1410-1436) and the closest-point kernel uses the segment [o, isect.p]
 * (photonbeam.cpp:499).
 *
 * Semantics are the reference's, bit for bit per (segment, beam) pair (see DESIGN.md "parity
 * contract"): candidate set = beams whose WorldBound box (group box for beams with identical
 * centroids) passes the gamma(3)-padded slab test; contribution 1e-5*powerEnd*sqrt(1-(d/(R+r))^2)
 * for d < R + r, no phase, no camera throughput.  Only the float summation order differs.
 *
 * Conventions: plain pointers and sizes; xyz arrays are interleaved float[3*n]; RGB arrays
 * float[3*n].  No exceptions cross the ABI; every call returns a bre_status and stores a message
 * retrievable with bre_last_error().  One context per GPU; a context is not thread-safe.
 * Errors follow pbrt's style of "report and continue" only in the sense that a failed call leaves
 * the context usable; no function aborts the process.
 */
#ifndef BRE_H
#define BRE_H

#include <stdint.h>

#include "bre_scene.h"

#ifdef __cplusplus
extern "C" {
#endif

#define BRE_ABI_VERSION 3 /* 2: triangle scene model (bre_scene.h); 3: multi-GPU entry points */

typedef struct bre_ctx bre_ctx;

typedef enum bre_status {
    BRE_OK = 0,
    BRE_ERR_INVALID_ARG = 1, /* null pointer, negative size, pixel index out of range ... */
    BRE_ERR_HIP = 2,         /* a HIP runtime call failed (message has the HIP error string) */
    BRE_ERR_OOM = 3,         /* device allocation failed */
    BRE_ERR_STATE = 4,       /* e.g. bre_gather before any bre_set_beams */
    BRE_ERR_NO_DEVICE = 5    /* no HIP device / bad device ordinal */
} bre_status;

/* Options for bre_set_option(). */
typedef enum bre_option {
    BRE_OPT_COUNTERS = 1,    /* 0/1: per-segment candidate / contribution / node-visit counting */
    BRE_OPT_TIMING = 2,      /* 0/1: HIP-event timing of build and gather kernels (bre_stats ms) */
    BRE_OPT_KERNEL = 3,      /* 0 = the production gather (default): wave-packet traversal over a tree
                                of BRE_OPT_TILE_LEAF-beam leaf tiles, packet bundle reject, per-lane
                                separable prefilter, wavefront-compacted exact stage.
                                4 = the same kernel on a tree of BRE_OPT_LEAF_SIZE-beam leaves,
                                2 = thread-per-segment traversal (an independent cross-check),
                                5 = capsule-chunk index.  Values 1, 3 and 6 (round-1 kernels) are
                                rejected.  Every kernel gives the same pair contributions. */
    BRE_OPT_LEAF_SIZE = 4,   /* beams per BVH leaf cluster, 1..64 (default 1); applies at next build */
    BRE_OPT_SQRT_MODE = 5,   /* 0 = libstdc++ reading of WorldBound's sqrt (double), 1 = float */
    BRE_OPT_SPLIT = 6,       /* kernels 0/4: BVH subtrees per segment packet, power of two 1..1024 (default 256) */
    BRE_OPT_PREFILTER = 7,   /* kernels 0/4/5: 0/1 conservative line-distance rejects before the exact
                                closest-point code (default 1; results are identical either way) */
    BRE_OPT_SHARD_RANK = 8,  /* camera pass: walk only the 16x16 pixel tiles (the reference's
                                camera-pass tiles, photonbeam.cpp:345-347) of the blocks of
                                BRE_OPT_SHARD_BLOCK^2 tiles whose row-major block index b has
                                b % count == rank (block 1: tile t with t % count == rank) */
    BRE_OPT_SHARD_COUNT = 9, /* camera pass: number of image-tile shards (default 1 = all tiles).
                                Set the count before the rank.  Per-pixel results do not depend on
                                the sharding, so summing the shards' Ld gives the 1-shard image. */
    BRE_OPT_TILE_LEAF = 10,  /* kernel 0: beams per leaf tile of its tree, 1..64
                                (default 64); applies at the next build */
    BRE_OPT_CHUNK_LEN = 11,  /* kernel 5: chunk length in units of E/100, E = (R + r)(1 + 1e-3) + margin
                                (25..100000, default 400) */
    BRE_OPT_CHUNK_LEAF = 12, /* kernel 5: chunks per LBVH leaf, 1..64 (default 1) */
    BRE_OPT_SORT_SEGMENTS = 13, /* bre_gather_camera: 0/1 hand the camera-pass segments to the gather
                                  in 6-D Morton order of (origin, end point) (default 1); pixel sums
                                  are the same pair contributions either way */
    BRE_OPT_SHARD_BLOCK = 14, /* tile shards: tiles per side of the blocks dealt to the shards; packet
                                shards: consecutive packets per chunk dealt to the shards (1..4096,
                                default 1) */
    BRE_OPT_SHARD_MODE = 15, /* 0 (default): shards own image tiles (SHARD_BLOCK), each pixel is written
                                by one shard.  1: PACKET shards -- every shard runs the whole camera
                                pass and gathers its round-robin share of the sorted 64-segment packets
                                (bre_shard_segments); the surface radiance of pixel p is added by shard
                                p % count; the shards' Ld films SUM to the whole film (a reduce).
                                2: WORK-ROOT shards -- every shard runs the whole camera pass and
                                gathers every segment against the BVH work roots rank, rank + count, ...
                                of the size-ordered list (kernels 0/4); surface radiance and films as
                                in 1, per-segment outputs are the shard's subtrees' partial sums */
    BRE_OPT_FILM_CLASSES = 16 /* 1 (default) or BRE_FILM_CLASSES (8): the films the camera pass and the
                                kernel 0 / 4 gathers add to are 8 planes of float[3*npix] -- class c
                                holds the surface radiance of the pixels p with p % 8 == c and the
                                gather terms of the segments in the sorted order's packet chunks k
                                (BRE_OPT_SHARD_BLOCK packets each) with k % 8 == c, each pixel's
                                segments of a class added in the caller's order.  The image is the sum
                                of the planes in class order (bre_resolve_classes).  Packet shard r of
                                count (count dividing 8) computes exactly classes c % count == r, so
                                gathering the shards' planes and resolving gives the 1-shard image
                                bit for bit (dist.py ShardedFrame, bench.py --gpus N).  The caller's
                                film buffers (bre_camera_pass d_surface, bre_gather_camera*,
                                bre_gather_device, bre_render_iteration) must then hold 8 * 3 * npix
                                floats; the entry points with films of their own (bre_gather,
                                bre_render, bre_render_progressive, bre_gather_sharded) refuse the
                                option with BRE_ERR_STATE. */
} bre_option;

#define BRE_FILM_CLASSES 8

typedef struct bre_stats {
    int64_t n_beams;         /* beams in the current set (after set_beams) */
    int64_t n_beams_valid;   /* beams with a finite WorldBound (zero-length beams have a NaN box) */
    int64_t n_nodes;         /* BVH interior nodes */
    int64_t n_segments;      /* segments in the last gather */
    int64_t candidates;      /* sum over segments of C = beams passing the reference box test
                                (= size of PhotonBeamBVH::Intersect's result); counters only */
    int64_t contributions;   /* pairs with d < R + r that added to the pixel; counters only */
    int64_t node_visits;     /* interior-node visits summed over waves (kernel 1) or threads
                                (kernel 2); counters only */
    int64_t leaf_visits;     /* kernel 1, counters: leaf clusters evaluated, per wave */
    int64_t beam_evals;      /* kernel 1, counters: beam records evaluated, per wave */
    int64_t ccp_wave_evals;  /* kernel 1, counters: exact closest-point executions, per wave */
    int64_t prefilter_rejects; /* kernel 1, counters: lane-level line-distance rejects */
    int64_t useful_beam_evals; /* counters: kernel 1 beam evaluations where >= 1 lane is a candidate; kernels 3/4: beams kept by the packet bundle test */
    int64_t max_stack_depth;   /* kernel 3, counters: deepest LDS node stack used by any wave */
    int64_t redo_items;        /* kernel 3, counters: (packet, subtree) items handed to kernel 1
                                  (incoherent packets or LDS-stack overflow) */
    double build_ms;         /* device time of the last BVH build (timing only) */
    double gather_ms;        /* device time of the last gather kernel (timing only) */
    int64_t n_photons;       /* photons traced by the last bre_trace_photons */
    double photon_ms;        /* device time of the last photon pass, both passes (timing only) */
    int64_t n_camera_segments; /* segments of the last bre_camera_pass */
    double camera_ms;        /* device time of the last camera pass incl. compaction (timing only) */
    int64_t n_chunks;        /* kernel 5: chunks in the index of the last gather */
    int64_t queued_pairs;    /* kernels 0/4: (segment, beam) pairs that passed the prefilters and ran the
                                exact stage (box test + ComputeClosestPoints); counted with counters,
                                and by the production instantiation itself whenever per-segment
                                counts are requested (read back with counters or timing on) */
} bre_stats;

/* ---- context ---- */
bre_status bre_create(int device, bre_ctx **out);
void bre_destroy(bre_ctx *ctx);
const char *bre_last_error(const bre_ctx *ctx);
int bre_abi_version(void);
bre_status bre_set_option(bre_ctx *ctx, int option, int64_t value);
/* Use an existing hipStream_t (cast to void*) for all work of this context; NULL = the
   context's own stream.  The caller keeps ownership of a stream it passes in.
   The photon pass (with its BVH build) and the camera pass run on an internal stream of the device's
   highest priority (internal option 117, on by default), forked from this stream -- the pass starts
   after everything queued on it before the call -- and joined back to it before the call returns, so
   work queued on this stream afterwards waits for the pass: stream order towards the caller is exactly
   as if the pass ran on this stream (tests/test_pass_stream_gpu.py reuses a freed film right after
   each pass, with the option on and off). */
bre_status bre_set_stream(bre_ctx *ctx, void *hip_stream);
bre_status bre_synchronize(bre_ctx *ctx);
bre_status bre_get_stats(const bre_ctx *ctx, bre_stats *out);

/* ---- beams (replaces `PhotonBeamBVH photonBeamBVH(std::move(photonBeams))`) ----
   start_xyz, end_xyz: float[3n]; radius: float[n]; power_end_rgb: float[3n].
   bre_set_beams copies host arrays; bre_set_beams_device reads device arrays (no copy kept:
   the build consumes them before returning control of the stream).  n = 0 clears the set
   (every gather then adds nothing, as an empty PhotonBeamBVH returns no beams). */
bre_status bre_set_beams(bre_ctx *ctx, int64_t n, const float *start_xyz, const float *end_xyz,
                         const float *radius, const float *power_end_rgb);
bre_status bre_set_beams_device(bre_ctx *ctx, int64_t n, const float *d_start_xyz,
                                const float *d_end_xyz, const float *d_radius,
                                const float *d_power_end_rgb);

/* ---- gather (replaces photonbeam.cpp:494-508 for every segment of an iteration) ----
   seg_o_xyz, seg_p_xyz, seg_d_xyz: float[3*nseg] (ray.o, isect.p, ray.d); seg_tmax: float[nseg]
   (ray.tMax); seg_pixel: int32[nseg], pixel index in [0, npix).
   accum_rgb: float[3*npix], accumulated (+=) like PhotonBeamPixel::Ld (may be NULL).  Kernels 0 / 4
   add deterministically: the per-segment sums are sorted by pixel (stable, so a pixel's segments
   keep the caller's order) and one thread per pixel adds its segments in that order, then adds the
   total to the pixel once.  That pass is O(segments) in all, but a pixel's run is serial: callers
   whose segments pile onto a few pixels (thousands per pixel) pay that run's length in one thread;
   camera-pass segments have at most maxdepth (+ null crossings) per pixel.
   seg_rgb: float[3*nseg] per-segment sums, overwritten (may be NULL).
   seg_counts: int32[2*nseg] per-segment {C candidates, contributions} (may be NULL).  With
   BRE_OPT_COUNTERS=1 both are counted (C by an extra box test of every visited beam); without it
   the production kernel counts the contributions alone, with its own control flow, and C = -1.
   beam_radius_cur: the integrator's currentBeamRadius R_cur.
   Device errors (a traversal-stack overflow: BRE_ERR_STATE; a seg_pixel outside [0, npix):
   BRE_ERR_INVALID_ARG) are never silent: an asynchronous call reports them at the context's next
   synchronising call (bre_synchronize, bre_gather, bre_trace_photons, bre_camera_pass, bre_get_*,
   bre_render*).
   bre_gather takes host pointers (PCIe copies in and out, synchronous); bre_gather_device
   takes device pointers and is asynchronous on the context's stream.  Both hand the segments to
   the production kernel in the coherence order of bre_gather_camera (BRE_OPT_SORT_SEGMENTS, kernels
   0 / 4) and scatter per-segment outputs back to the caller's order; under BRE_OPT_SHARD_MODE 1 with
   a shard count > 1 they gather only this shard's packets of that order (the other entries of the
   per-segment outputs are zeroed), exactly as bre_gather_camera does. */
bre_status bre_gather(bre_ctx *ctx, int64_t nseg, const float *seg_o_xyz, const float *seg_p_xyz,
                      const float *seg_d_xyz, const float *seg_tmax, const int32_t *seg_pixel,
                      float beam_radius_cur, int64_t npix, float *accum_rgb, float *seg_rgb,
                      int32_t *seg_counts);
bre_status bre_gather_device(bre_ctx *ctx, int64_t nseg, const float *d_seg_o_xyz,
                             const float *d_seg_p_xyz, const float *d_seg_d_xyz,
                             const float *d_seg_tmax, const int32_t *d_seg_pixel,
                             float beam_radius_cur, int64_t npix, float *d_accum_rgb,
                             float *d_seg_rgb, int32_t *d_seg_counts);

/* The image of BRE_OPT_FILM_CLASSES films: out[i] = classes[0][i] + ... + classes[7][i] for the
   3*npix floats i, added in class order (device pointers; asynchronous on the context's stream).
   out may alias classes[0]. */
bre_status bre_resolve_classes(bre_ctx *ctx, int64_t npix, const float *d_classes, float *d_out);

/* The render's film over iterations: d_dst[i] += d_src[i] for the n_floats floats i, then d_src[i] = 0
   when clear_src is nonzero (device pointers, distinct; asynchronous on the context's stream).  The
   reference adds every iteration into the same PhotonBeamPixel::Ld (photonbeam.cpp:477-504, 578); a
   caller that renders each iteration into its own image (bench.py's pipelined contexts) adds it with
   this one-wave kernel, which -- unlike a framework's multi-wave elementwise kernels -- runs beside a
   concurrent gather of the other context instead of after it. */
bre_status bre_film_add(bre_ctx *ctx, int64_t n_floats, float *d_src, float *d_dst, int32_t clear_src);
/* Pipelined contexts on one device (NULL clears): every later gather of ctx starts its tile kernel only
   after prev's last tile kernel has finished (an event wait on ctx's stream right before the launch).
   The segment sort and the other preparation of ctx's gather, and its passes, still run beside prev's
   gather; only the two tile kernels do not interleave -- their one-wave workgroups would otherwise share
   the CUs and the L2 two trees at a time (round 6, profiles/r6).  bre_destroy(prev) unlinks ctx (its
   later gathers no longer wait). */
bre_status bre_set_gather_after(bre_ctx *ctx, bre_ctx *prev);
/* Timing (NULL, NULL clears): every later gather of the tile kernels (kernels 0 / 4) records the caller's
   hipEvent_t start_event on the context's stream right before its first tile-kernel launch (after any
   bre_set_gather_after wait) and end_event right after its last one, so their elapsed time is the tile
   kernel alone -- not the segment sort before it, the per-segment reduce and film compose after it, or
   the wait for a pipelined context's gather. */
bre_status bre_set_gather_events(bre_ctx *ctx, void *start_event, void *end_event);

/* ---- multi-GPU gather (SURVEY.md §8(b) `bre_gather_sharded`, §8(e)) ----
   ctxs[0 .. n_ctx): one context per GPU (several contexts on one device are allowed: tests), each
   driven by its own host thread for the duration of the call.  The reference renders in one
   process over a thread pool (photonbeam.cpp:444-557); this is the same batched gather split over
   devices with the photon map replicated.
   bre_set_beams_sharded: bre_set_beams on every context, in parallel (the same beam set and BVH on
   every device).
   bre_gather_sharded: bre_gather semantics for host segments.  Context i gathers packet shard i of
   n_ctx of the coherence-sorted segment order (BRE_OPT_SHARD_MODE 1, BRE_OPT_SHARD_BLOCK 1; each
   context's own shard options are restored afterwards), so every device gets the same mix of cheap
   and costly packets.  The devices' films are summed on the host in context order and added (+=)
   into accum_rgb; per-segment outputs (each entry is gathered by exactly one context) are merged the
   same way.  The first failing context's status is returned, its message prefixed with the context
   index in bre_last_error(ctxs[0]). */
bre_status bre_set_beams_sharded(bre_ctx *const *ctxs, int n_ctx, int64_t n, const float *start_xyz,
                                 const float *end_xyz, const float *radius, const float *power_end_rgb);
bre_status bre_gather_sharded(bre_ctx *const *ctxs, int n_ctx, int64_t nseg, const float *seg_o_xyz,
                              const float *seg_p_xyz, const float *seg_d_xyz, const float *seg_tmax,
                              const int32_t *seg_pixel, float beam_radius_cur, int64_t npix, float *accum_rgb,
                              float *seg_rgb, int32_t *seg_counts);

/* ---- photon pass (replaces photonbeam.cpp:362-437: emission, TracePhotonBeamRecursive and the
   merge into one beam vector, then the PhotonBeamBVH build of :438) ----
   Traces photons [0, n_photons) of `iteration` on the device (photon i uses PCG32 sequence
   iteration*n_photons + i + 1, :386-389), keeps the beams on the device in the reference's order
   (photon-major, push order within a photon) and builds the BVH over them, exactly as
   bre_set_beams would with the same arrays.  max_depth in [1, BRE_MAX_DEPTH]; beam_radius is the
   iteration's currentBeamRadius.  *n_beams (may be NULL) receives the beam count.  Synchronous. */
bre_status bre_trace_photons(bre_ctx *ctx, const bre_scene *scene, int64_t n_photons, int32_t iteration,
                             int32_t max_depth, float beam_radius, int64_t *n_beams);
/* Copy the current beam set (from bre_set_beams or bre_trace_photons) back to host arrays in
   their original order; at most `capacity` beams are written, *n_beams receives the set size.
   BRE_ERR_STATE after bre_set_beams_device (the library keeps no copy of caller device arrays). */
bre_status bre_get_beams(bre_ctx *ctx, int64_t capacity, float *start_xyz, float *end_xyz, float *radius,
                         float *power_end_rgb, int64_t *n_beams);

/* ---- camera pass (replaces photonbeam.cpp:444-555 up to the gather) ----
   Walks one camera path per pixel of a width x height film for `iteration` on the device
   (HaltonSampler sample `iteration` of each pixel, perspective pinhole, scene intersection,
   homogeneous-medium transmittance, Lambertian bounces and Russian roulette) and keeps the
   segment [ray.o, isect.p] of every surface-hit camera ray in the context: depth-major, pixels in
   8x8-tile order within a depth.  d_surface_rgb (device float[3*W*H], may be NULL) receives += the
   surface radiance of rendersurfaces (emission seen directly + UniformSampleOneLight).  max_depth
   in [1, BRE_MAX_DEPTH].  *n_segments (may be NULL) receives the segment count.  Synchronous. */
bre_status bre_camera_pass(bre_ctx *ctx, const bre_scene *scene, int32_t width, int32_t height, int32_t iteration,
                           int32_t max_depth, int32_t render_surfaces, int32_t render_media, float *d_surface_rgb,
                           int64_t *n_segments);
/* Gather the context's camera segments against its beam set: bre_gather_device on them, adding
   into d_accum_rgb (device float[3*W*H] of the last camera pass).  Asynchronous. */
bre_status bre_gather_camera(bre_ctx *ctx, float beam_radius_cur, float *d_accum_rgb);
/* bre_gather_camera with per-segment outputs in the camera-pass order of bre_get_segments:
   d_seg_rgb (device float[3*n], may be NULL), d_seg_counts (device int32[2*n], may be NULL; as
   bre_gather's seg_counts).  The gather itself runs exactly as in bre_gather_camera (the same
   coherence order and kernel instantiation); only the outputs are scattered back.  Asynchronous. */
bre_status bre_gather_camera_segments(bre_ctx *ctx, float beam_radius_cur, float *d_accum_rgb, float *d_seg_rgb,
                                      int32_t *d_seg_counts);
/* Copy the camera segments back (tests): xyz arrays, tmax, pixel index and path depth. */
bre_status bre_get_segments(bre_ctx *ctx, int64_t capacity, float *o_xyz, float *p_xyz, float *d_xyz, float *tmax,
                            int32_t *pixel, int32_t *depth, int64_t *n_segments);

/* ---- the integrator (PhotonBeamIntegrator::Render, photonbeam.cpp:329-586) ----
   For iteration in [start_iteration, end_iteration): photon pass (bre_trace_photons) with the
   iteration's radius R_i, BVH build, camera pass, gather of every segment with R_i into the
   per-pixel Ld (device, float[3*W*H], accumulated across calls: the caller zeroes it once), then
   R_{i+1} = R_i (i + alpha) / (i + 1).  bre_render_iteration runs one iteration on caller device
   memory; bre_render runs the whole range and writes L = Ld / end_iteration (the image the
   reference hands to Film::SetImage at its last write, :565-583) to host image_rgb[3*W*H]. */
bre_status bre_render_iteration(bre_ctx *ctx, const bre_scene *scene, const bre_render_params *params,
                                int32_t iteration, float *d_ld_rgb);
bre_status bre_render(bre_ctx *ctx, const bre_scene *scene, const bre_render_params *params, float *image_rgb);
/* The write schedule of Render (photonbeam.cpp:564-584): after iteration `iter`, when
   iter + 1 == end_iteration or (iter + 1) % write_frequency == 0, the image L = Ld / (iter + 1)
   (host float[3*W*H], row-major from the top row, valid only during the call) is handed to
   `on_image(iter, L, user)`, where the reference calls Film::SetImage + Film::WriteImage.
   As in the reference, a negative write_frequency -k also fires every k iterations; INT32_MIN (the
   reference's default 1 << 31 after wrapping) never divides iter + 1, and 0 means "only at the end".  A non-zero return from on_image stops the render with
   BRE_ERR_STATE.  on_image may be NULL. */
typedef int (*bre_image_fn)(int32_t iteration, const float *image_rgb, void *user);
bre_status bre_render_progressive(bre_ctx *ctx, const bre_scene *scene, const bre_render_params *params,
                                  int32_t write_frequency, bre_image_fn on_image, void *user);

/* ---- integrator helpers (photonbeam.cpp:354-356, 562, 578) ---- */
/* R_i for iteration i: R_{k+1} = R_k * (k + alpha) / (k + 1), R_0 = initial, in float. */
float bre_beam_radius_at(float initial_radius, float alpha, int iteration);
/* How many of n_segments camera segments shard `rank` of `count` gathers under BRE_OPT_SHARD_MODE 1:
   the (sorted) order's 64-segment packets form chunks of `chunk` consecutive packets (the context's
   BRE_OPT_SHARD_BLOCK), dealt round-robin -- chunk c to shard c % count -- so every shard gets the same
   mix of cheap primary and costly bounce packets while its concurrent packets stay neighbours. */
int64_t bre_shard_segments(int64_t n_segments, int32_t rank, int32_t count, int32_t chunk);
/* image = Ld / (iter + 1) for npix pixels (host arrays). */
bre_status bre_resolve_image(int64_t npix, const float *ld_rgb, int iteration, float *out_rgb);

/* ---- device self-check (tests) ----
   Runs libbre's own device copies of the scalar primitives the passes and the gather share on n host
   inputs x (synchronous; y is host memory):
     kind 0: NextFloatUp(x)   1: NextFloatDown(x)   (pbrt.h:215-239; OffsetRayOrigin, geometry.h:1438-1458)
     kind 2: y[2i] = the exact stage's square root (bre_math.h sqrt_cr_noscale), y[2i+1] = sqrtf(x)
     kind 3: FindInterval(n_aux, [&](int k) { return aux[k] <= x; }) as a float (pbrt.h:377-389; the
             light choice of Distribution1D::SampleDiscrete, sampling.h:90-100)
     kind 4: y[2i] = x / aux[0] by the exact stage's shared-reciprocal division (div_by_shared),
             y[2i+1] = x / aux[0] correctly rounded
     kind 5: the tile kernel's S = aux[0] work roots (k_roots) of the binary tree whose n / 16 Node
             records (bre_device.h: only child[2] and nleaf are read) are x's words; y receives S + 1
             int32 words: the roots largest first (kEmptyChild-padded), then their count
     kind 6 / 8: the pass chain's stable radix sort (bre_slot.hip) of the n / 2 64-bit (kind 8: n 32-bit)
             keys in x by bits [aux[0], aux[1]), the values being the input positions; y receives the
             sorted keys, then the values (int32)
     kind 7: its exclusive scan of the n int32 words of x; y receives n + 1 int64 (the total last)
     kind 9: y[4i .. 4i + 3] = expf, logf, sinf, cosf of x[i] as the photon and camera passes compute
             them (include/bre_fmath.h: the x86-64 glibc libm's results bit for bit)
   so the tests can hold them against the reference's own primitive tests (src/tests/fp_tests.cpp,
   find_interval.cpp) and against the compiler's correctly rounded sqrt and division. */
bre_status bre_device_check(bre_ctx *ctx, int32_t kind, int64_t n, const float *x, int32_t n_aux, const float *aux,
                            float *y);

#ifdef __cplusplus
}
#endif
#endif /* BRE_H */
