#!/usr/bin/env python3
"""Benchmark: beam-radiance estimates/sec at 1M photons (BASELINE.json metric), MI355X.

Default workload `c2` = BASELINE.json configs[1] / SURVEY.md §8d C2: the Cornell box in homogeneous
fog (sigma_a 0.05, sigma_s 0.5, g 0), 512x512 film, 1,000,000 photons per iteration, maxdepth 5,
initialbeamradius 0.01, alpha 0.5, 16 iterations (16 spp).  One *step* is one full iteration of
PhotonBeamIntegrator::Render (photonbeam.cpp:362-562) on the GPU, everything resident in HBM:
photon pass (emission + TracePhotonBeamRecursive, ~2.7M beams) + BVH build + camera pass + the
gather of every camera segment into the pixels' Ld.  One *estimate* = the full gather for one
camera segment (photonbeam.cpp:494-508).  value = segments gathered by all ranks / max-rank wall
time of the timed steps.  Iteration k of the timed loop is the reference's iteration k (radius
schedule and sampler indices included), so `--steps 16` is exactly the C2 render.

Multi-GPU (`--gpus N`): one process per GPU.  Launched by torch.distributed.run (WORLD_SIZE set) it
joins that group; launched alone with N > 1 it starts N rank processes itself (a torch.distributed.run
child, before any GPU call) and exits with its status.  Default scaling is STRONG: one film (the
workload's W x H); every rank traces the same photons (per-photon PCG32 sequences, no communication),
builds its own BVH, runs the whole camera pass and sorts all segments, then gathers its round-robin
share of the sorted 64-segment packets (`--shard-mode packets`, libbre BRE_OPT_SHARD_MODE 1: exactly the
single-GPU packets, every rank the same mix); the partial films are summed to rank 0 once per written image
(the last step), one RCCL reduce.  `--shard-mode tiles` deals the reference's 16x16 tiles
(photonbeam.cpp:345-347) instead, in blocks of `--shard-block`^2, with one RCCL gather of the owned
pixel bands.  `--scaling weak` gives every rank its own film of the same size (N independent renders).
`--emulate-shard R/N` runs rank R's share of an N-GPU strong-scaling run alone on one GPU.

Also reported (rank 0, N = 1):
* `roofline` — the tile kernel's VALU issue roofline (`bound` "valu_issue"): wave64 VALU
  instructions per second of the iteration-0 launch against 256 CU x 4 SIMD / 2 clocks, from this
  run's own rocprofv3 PMC passes (`issue`: SQ counters, LDS busy, waits, and the vector-memory
  path's TA / TD busy fractions with the busiest unit named -- since round 3 the TD data-return
  path); `traffic` = HBM bytes per
  launch from the same passes (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE).  `hbm`: the
  requested bytes per launch (node and beam lines of the visited tiles, the segments, the exact
  stage's 112 B per queued pair, the partial sums; counted live by the counter pass) / the launch's
  HIP-event time against 8 TB/s, and the measured HBM traffic against it.  Without rocprofv3 the
  line falls back to `bound` "hbm" on the requested bytes.  The SURVEY §8d reference-tree byte
  model is kept as `ref_model_*` (not a fraction: one staged beam line feeds 64 lanes).
* `cpu_baseline` — the oracle's CPU restatement of the reference algorithm (SAH tree, per-query
  vector<shared_ptr>, all host threads, plus 1 thread), timed on bounded samples of the same
  segments and beams at the first and last timed iterations.
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
NODE4_BYTES = 128.0     # one visit of the tile kernel's 4-wide walk reads one Node4 record (bre_device.h)
CUS, SIMDS = 256, 4     # VALU issue peak: one wave64 instruction per 2 clocks per SIMD-32


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed iterations (default: c2 16 = the whole 16-spp render, c5 10 passes, else 4)")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c2",
                    help="BASELINE.json configs[1..4] (SURVEY.md §8d), c4-1m (the 2K tiled film at C2's 1M "
                         "photons), or the kernel-only synthetic set")
    ap.add_argument("--photons", type=int, default=None, help="photons per iteration")
    ap.add_argument("--beams", type=int, default=1_000_000, help="synthetic: beams")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--scaling", choices=["weak", "strong"], default="strong",
                    help="strong (default): one film split by 16x16 tiles over the N GPUs; weak: a film per GPU")
    ap.add_argument("--grid-n", type=int, default=64, help="c3/c5: smoke density grid resolution")
    ap.add_argument("--radius", type=float, default=0.01, help="initialbeamradius (scenes) / R (synthetic)")
    ap.add_argument("--alpha", type=float, default=0.5)
    ap.add_argument("--max-depth", type=int, default=5)
    ap.add_argument("--kernel", type=int, default=0)
    ap.add_argument("--leaf-size", type=int, default=1)
    ap.add_argument("--split", type=int, default=256, help="BVH subtrees (work roots) per segment packet")
    ap.add_argument("--prefilter", type=int, default=1)
    ap.add_argument("--chunk-len", type=int, default=400, help="kernel 5: chunk length in units of E/100")
    ap.add_argument("--chunk-leaf", type=int, default=1, help="kernel 5: chunks per LBVH leaf")
    ap.add_argument("--sort-segments", type=int, default=1, help="coherence-sort the camera segments (0/1)")
    ap.add_argument("--occupancy", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--tile-leaf", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--sort-key", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--block-map", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--tscan", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--beam-key", type=int, default=-1, help=argparse.SUPPRESS)  # tree build key study (option 110)
    ap.add_argument("--margin", type=int, default=-1, help=argparse.SUPPRESS)  # prefilter margin A/B (option 111)
    ap.add_argument("--tile-axis", type=int, default=-1, help=argparse.SUPPRESS)  # tile line reject A/B (option 112)
    ap.add_argument("--split-records", type=int, default=-1, help=argparse.SUPPRESS)  # BeamRec layout A/B (option 113)
    ap.add_argument("--film-compose", type=int, default=-1, help=argparse.SUPPRESS)  # film accumulation A/B (option 114)
    ap.add_argument("--photon-single", type=int, default=-1, help=argparse.SUPPRESS)  # photon pass form A/B (option 116)
    ap.add_argument("--pass-priority", type=int, default=-1, help=argparse.SUPPRESS)  # option 117 A/B
    ap.add_argument("--partial-mib", type=int, default=-1, help=argparse.SUPPRESS)  # option 109: launches per gather
    ap.add_argument("--readback", type=int, default=-1, help=argparse.SUPPRESS)  # option 118 A/B
    ap.add_argument("--slot-passes", type=int, default=-1, help=argparse.SUPPRESS)  # option 119 A/B
    ap.add_argument("--coarse-keys", type=int, default=-1, help=argparse.SUPPRESS)  # option 121 A/B
    ap.add_argument("--film-classes", type=int, default=1,
                    help="packet shards: keep the film as 8 packet-class planes, gathered and resolved in class "
                         "order, so every N dividing 8 renders the one-GPU film bit for bit (0: one film, "
                         "sum-reduced)")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="scenes: two libbre contexts on two streams, iteration k+1's photon pass / build / "
                         "camera pass overlapping iteration k's gather (0: one context)")
    ap.add_argument("--gather-fence", type=int, default=1,
                    help="pipelined contexts: 1 = a context's tile kernel waits for the other's last one "
                         "(bre_set_gather_after), 0 = the two gathers may interleave")
    ap.add_argument("--gather-priority", type=int, default=0, help=argparse.SUPPRESS)  # study: context 0 high priority
    ap.add_argument("--shard-mode", choices=["packets", "tiles", "roots"], default="packets",
                    help="strong scaling: each GPU gathers a range of the sorted segment packets (default) "
                         "or owns image tiles")
    ap.add_argument("--shard-block", type=int, default=1,
                    help="tile shards: tiles per side of the image blocks dealt round-robin to the GPUs")
    ap.add_argument("--emulate-shard", type=str, default=None, help=argparse.SUPPRESS)  # "R/N": rank R's share on 1 GPU
    # rehearsal of the N-rank flow on a one-GPU box: every rank on cuda:0, collectives over gloo
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl", help=argparse.SUPPRESS)
    ap.add_argument("--share-gpu", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline gather time (all threads)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-diag", action="store_true", help="skip the untimed counters/timing pass (profiling runs)")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 PMC passes of the roofline")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--segment-kind", choices=["camera", "bounce"], default="camera",
                    help="synthetic: camera primary segments or incoherent bounce segments")
    ap.add_argument("--entry", choices=["camera", "boundary"], default="camera",
                    help="camera (default): the in-library camera pass hands its segments to bre_gather_camera; "
                         "boundary: the same segments in the reference's recorder order (16x16 tiles dealt to 16 "
                         "threads, each pixel's depths in order) through bre_gather_device, the C-ABI entry the "
                         "pbrt adapter uses")
    ap.add_argument("--no-legs", action="store_true",
                    help="c2: skip the untimed-by-headline C3 (N=1), C4 and C5 (every N) legs")
    ap.add_argument("--c4-leg", choices=["auto", "on", "off"], default="auto",
                    help="c2: the C4 iteration-0 gather leg (auto: with strong scaling, at every N)")
    ap.add_argument("--c5-leg", choices=["auto", "on", "off"], default="auto",
                    help="c2: the C5 last-pass (iteration 9) gather leg (auto: with strong scaling, at every N)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--progress", action="store_true",
                    help="print a line per timed step to stderr (synchronises each step; long C4/C5 runs)")
    a = ap.parse_args(argv)
    preset = WORKLOADS[a.workload]
    for k in ("steps", "photons", "width", "height"):
        if getattr(a, k) is None:
            setattr(a, k, preset[k])
    return a


# BASELINE.json configs[1..4].  c4/c5 are 8-GPU configurations: at N=1 they run as
# stated (long) unless --photons / --width / --height scale them down.  c4-1m is the 2K tiled film
# at C2's photon count (the scaling study that fits one GPU's time budget).
WORKLOADS = {
    "c2": dict(steps=16, photons=1_000_000, width=512, height=512, medium="fog", g=0.0),
    "c3": dict(steps=4, photons=5_000_000, width=1024, height=1024, medium="smoke", g=0.7),
    "c4": dict(steps=4, photons=20_000_000, width=2048, height=2048, medium="fog", g=0.0),
    "c4-1m": dict(steps=4, photons=1_000_000, width=2048, height=2048, medium="fog", g=0.0),
    "c5": dict(steps=10, photons=50_000_000, width=1024, height=1024, medium="smoke", g=0.7),
    "synthetic": dict(steps=10, photons=0, width=512, height=512, medium="fog", g=0.0),
}

KERNEL_NAMES = {0: "kernel 0: wave packets over 64-beam leaf tiles, packet bundle reject, separable per-lane "
                   "prefilter, wavefront-compacted exact stage",
                2: "kernel 2: thread-per-segment", 4: "kernel 4: tile kernel on BRE_OPT_LEAF_SIZE leaves",
                5: "kernel 5: capsule-chunk index"}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(args) -> int:
    """--gpus N > 1 without a process group: start N ranks (torch.distributed.run, one per GPU) as a
    child process — nothing here has touched the GPU — and return its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    import torch
    import torch.distributed as dist

    bre = importlib.import_module("beam-radiance-estimate-pbrt_amd")
    dmod = importlib.import_module("beam-radiance-estimate-pbrt_amd.dist")

    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if env_world > 1:
        if args.share_gpu:
            local = 0
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
        world, rank = dist.get_world_size(), dist.get_rank()  # n_gpus from the live process group
    else:
        torch.cuda.set_device(0)
        world, rank = 1, 0
    if args.gpus != world and rank == 0:
        print(f"bench.py: --gpus {args.gpus} but the process group has {world} ranks; reporting {world}",
              file=sys.stderr)
    dev = torch.device("cuda", local if world > 1 else 0)

    strong = args.scaling == "strong"
    srank, scount = (rank, world) if strong else (0, 1)
    if args.emulate_shard and world == 1:  # one rank's share of an N-GPU strong-scaling run, on this GPU
        srank, scount = (int(x) for x in args.emulate_shard.split("/"))
    classes = film_classes(args)
    frame = dmod.ShardedFrame(args.width, args.height, srank, scount, device=dev, block=args.shard_block,
                              packets=args.shard_mode == "packets", roots=args.shard_mode == "roots",
                              classes=classes)
    def make_ctx(priority=0):
        return make_context(bre, args, dev, priority)

    # --gather-priority 1: the first context's stream at a higher priority than the second's (study)
    g, stream = make_ctx(-1 if args.gather_priority else 0)
    torch.cuda.set_stream(stream)

    if args.workload != "synthetic":
        # --pipeline 1: a second context on a second stream, iterations alternating between them, so
        # iteration k+1's photon pass, BVH build and camera pass overlap iteration k's gather
        extra = [make_ctx()] if (args.pipeline and not args.pmc_child) else []
        if extra and args.gather_fence:
            # the two contexts' tile kernels back to back (bre_set_gather_after): each context's passes and
            # segment sort run inside the other's gather, but the gathers do not interleave
            extra[0][0].set_gather_after(g)
            g.set_gather_after(extra[0][0])
        wl = SceneWorkload(args, bre, [(g, stream)] + extra, frame, srank, scount)
    else:
        wl = SyntheticWorkload(args, bre, g, frame, dev)

    if args.pmc_child:  # one untimed iteration for the parent's rocprofv3 PMC pass
        wl.step(0, None, scratch=True)
        g.synchronize()
        g.close()
        return

    for k in range(args.warmup):
        wl.step(k, None, scratch=True)
    torch.cuda.synchronize(dev)

    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    for a_, b_ in events:  # create the HIP events (torch makes them on first record) before libbre records them
        a_.record()
        b_.record()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    nseg_local = 0
    for k in range(args.steps):
        nseg_local += wl.step(k, events[k], scratch=False)
        if args.progress:
            torch.cuda.synchronize(dev)
            print(f"bench.py: rank {rank} step {k + 1}/{args.steps} done at {time.perf_counter() - t0:.1f} s",
                  file=sys.stderr, flush=True)
        if k == args.steps - 1:
            wl.finish()  # the pipeline's second film into the frame
            if strong and world > 1:
                frame.gather_to_root(0)  # one RCCL reduce / gather per written image
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    # the rendered film's bits (root): with packet-class films the same for every N dividing 8
    digest = film_digest(frame) if (rank == 0 and args.workload != "synthetic" and not args.emulate_shard) else None
    gather_per_step = [a.elapsed_time(b) for a, b in events]
    gather_ms = float(np.mean(gather_per_step))
    if world > 1:
        cdev = dev if args.dist_backend == "nccl" else torch.device("cpu")
        tt = torch.tensor([elapsed, gather_ms], dtype=torch.float64, device=cdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, gather_ms = float(tt[0]), float(tt[1])
        tot = torch.tensor([nseg_local], dtype=torch.int64, device=cdev)
        dist.all_reduce(tot)
        total_seg = int(tot.item())
    else:
        total_seg = nseg_local
    value = total_seg / elapsed

    # untimed: one more step with counters and per-phase HIP-event timing inside libbre, at iteration 0
    # (the largest radius: the roofline's launch) and at the smallest-radius iteration the line times
    # (the scan-bound end of the render: C2 iteration 15 whenever --steps >= 16)
    diag, st, st_last = {}, None, None
    if not args.no_diag:
        g.set_option(bre.OPT_COUNTERS, 1)
        g.set_option(bre.OPT_TIMING, 1)
        diag = wl.diagnostics(0)
        st = g.stats()
        k_last = late_step(wl, args.steps)
        if getattr(wl, "iteration", None) and wl.iteration(k_last) != wl.iteration(0):
            d_last = wl.diagnostics(k_last)
            st_last = g.stats()
            st_last["_iteration"] = wl.iteration(k_last)
            st_last["_gather_ms"] = d_last.get("gather_ms_iter0")
        g.set_option(bre.OPT_COUNTERS, 0)
        g.set_option(bre.OPT_TIMING, 0)

    result = {
        "metric": ("beam-radiance estimates/sec at 1M photons" if args.photons in (0, 1_000_000) else
                   f"beam-radiance estimates/sec at {args.photons / 1e6:g}M photons"),
        "value": value,
        "unit": "estimates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "fp32",
        "data": wl.data,
        "config": wl.config(world),
        "film_digest": digest,
        "estimates_per_step_per_gpu": nseg_local / args.steps,
        "gather_kernel_ms": gather_ms,
        "gather_ms_per_step": gather_per_step if rank == 0 else None,
    }
    if st is not None:
        result.update(counter_block(st, args))
        result["candidate_pair_tests_per_s"] = result["candidates_per_estimate"] * value
    if st_last is not None:
        # the same counter block at the smallest-radius timed iteration (the late
        # iterations are scan-bound and their funnel belongs in the line)
        last = counter_block(st_last, args)
        last.update({"iteration": st_last["_iteration"], "gather_ms": st_last["_gather_ms"]})
        result["counters_last_iteration"] = last
    result.update(diag)

    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(wl, args, gather_per_step)
        result["cpu_baseline"] = cpu["report"]
        result["speedup_vs_cpu"] = value / cpu["report"]["value"]
    else:
        cpu = None
    if rank == 0 and world == 1 and st is not None:
        pmc = None if args.no_pmc else pmc_passes(args)
        # the counter pass and the PMC passes run iteration 0: hold its bytes to timed iteration 0's
        # HIP-event launch time (the average over the timed launches is gather_kernel_ms)
        result["roofline"] = roofline(st, args, wl, gather_per_step[0], pmc, cpu)
    wl.close()
    g.close()
    # the other BASELINE configurations, outside the headline's timed region: C3's
    # iteration 0 on rank 0 at N = 1, and C4's iteration-0 gather on every rank (max over ranks), so an
    # N-GPU run also measures the north star's scaling configuration
    if args.workload == "c2" and not args.no_legs and not args.emulate_shard:
        legs = {}
        if world == 1 and rank == 0:
            legs["c3"] = config_leg(args, bre, dmod, dev, "c3", 1, 0)
        if args.c4_leg == "on" or (args.c4_leg == "auto" and args.scaling == "strong"):
            legs["c4"] = config_leg(args, bre, dmod, dev, "c4", world, rank)
        if args.c5_leg == "on" or (args.c5_leg == "auto" and args.scaling == "strong"):
            # C5's last progressive pass (iteration 9: the smallest radius of its ten)
            legs["c5"] = config_leg(args, bre, dmod, dev, "c5", world, rank, iteration=9)
        if rank == 0:
            result["config_legs"] = legs
    if rank == 0:
        line = json.dumps(result)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.destroy_process_group()


def film_classes(args):
    """Packet-class films (libbre BRE_OPT_FILM_CLASSES, dist.ShardedFrame classes): on with packet
    shards (the default), so the N-GPU film is the one-GPU film bit for bit for every N dividing 8."""
    return 8 if (args.shard_mode == "packets" and args.film_classes and args.workload != "synthetic") else 1


def film_digest(frame):
    """sha256 of the resolved film's float32 bits and the film's sum (what the root holds after the
    timed steps): equal digests across N = 1, 2, 4, 8 show the split changes no bit."""
    import hashlib

    img = frame.resolve().detach().to("cpu").contiguous().numpy()
    return {"sha256": hashlib.sha256(img.tobytes()).hexdigest()[:32], "sum": float(img.astype(np.float64).sum()),
            "classes": frame.classes, "pixels": int(img.shape[0])}


def late_step(wl, steps):
    """The timed step of the smallest radius: the largest iteration the line times (C2 iteration 15
    whenever --steps >= 16; the last step when the workload has no iteration schedule)."""
    if not getattr(wl, "iteration", None):
        return steps - 1
    return max(range(steps), key=lambda k: (wl.iteration(k), -k))


def config_leg(args, bre, dmod, dev, name, world, rank, iteration=0):
    """One iteration of BASELINE configuration `name` on a fresh context (iteration 0, the largest radius,
    for C3 / C4; C5's last pass, iteration 9, the smallest radius of its progressive schedule): photon
    pass + build, camera pass, and the gather of this rank's share of the sorted segment packets, the
    gather timed by HIP events on its stream.  With N ranks: the gather time is the max over ranks (every
    rank's time is listed too), the estimates their sum, and the ranks' packet-class film planes are
    gathered to rank 0, whose film digest must not depend on N (the one-GPU film bit for bit).  Errors
    are reported in the leg, never raised (the headline line stands on its own)."""
    import argparse as ap_
    import torch
    import torch.distributed as dist

    try:
        a = ap_.Namespace(**vars(args))
        preset = WORKLOADS[name]
        a.workload, a.photons, a.width, a.height, a.steps = name, preset["photons"], preset["width"], preset["height"], 1
        a.entry, a.shard_mode = "camera", "packets"
        frame = dmod.ShardedFrame(a.width, a.height, rank, world, device=dev, block=1, packets=True,
                                  classes=film_classes(a))
        c, st = make_context(bre, a, dev)
        wl = SceneWorkload(a, bre, [(c, st)], frame, rank, world)
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
        ev[1].record()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        n = wl.step(iteration, ev, scratch=False)
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
        gms = ev[0].elapsed_time(ev[1])
        nb = int(wl.nbeams)
        per_rank, n_ranks = [gms], 1
        if world > 1:
            cdev = dev if args.dist_backend == "nccl" else torch.device("cpu")
            mine = torch.tensor([gms, wall, float(n)], dtype=torch.float64, device=cdev)
            parts = [torch.zeros_like(mine) for _ in range(world)]
            dist.all_gather(parts, mine)
            per_rank = [float(p[0]) for p in parts]
            gms, wall = max(per_rank), max(float(p[1]) for p in parts)
            n_all = int(sum(float(p[2]) for p in parts))
            n_ranks = dist.get_world_size()
            frame.gather_to_root(0)
            torch.cuda.synchronize(dev)
        else:
            n_all = n
        digest = film_digest(frame) if rank == 0 else None
        wl.close()
        c.close()
        it = wl.iteration(iteration)
        return {"workload": f"{name.upper()} iteration {it} ({preset['photons'] / 1e6:g}M photons, {a.width}x{a.height}, "
                            f"{'grid-density smoke, g 0.7' if preset['medium'] == 'smoke' else 'homogeneous fog'}, "
                            f"R {wl.radius(it):.6g})",
                "iteration": it, "n_gpus": world, "ranks_live": n_ranks, "estimates": n_all, "beams": nb,
                "gather_ms": gms, "gather_ms_per_rank": per_rank, "gather_estimates_per_s": n_all / (gms * 1e-3),
                "iteration_ms": wall * 1e3, "iteration_estimates_per_s": n_all / wall,
                "film_digest": digest,
                "timing": "gather: HIP events around the tile kernel launch on its stream, max over ranks (each "
                          "rank's in gather_ms_per_rank); iteration: wall time of photon pass + build + camera pass "
                          "+ gather, max over ranks; film_digest: the root's film after the plane gather (the same "
                          "for every N dividing 8)"}
    except Exception as e:  # reported, never fatal to the headline line
        return {"error": f"{type(e).__name__}: {e}"}


def make_context(bre, args, dev, priority=0):
    """One libbre context with the bench's options, on its own torch stream (the HIP events that time
    the gather are recorded on the stream the kernel runs on).  Returns (context, stream)."""
    import torch

    c = bre.BeamGather(dev.index, kernel=args.kernel, leaf_size=args.leaf_size, split=args.split,
                       prefilter=bool(args.prefilter))
    c.set_option(bre.OPT_SORT_SEGMENTS, args.sort_segments)
    if args.kernel == 5:
        c.set_option(bre.OPT_CHUNK_LEN, args.chunk_len)
        c.set_option(bre.OPT_CHUNK_LEAF, args.chunk_leaf)
    for opt, val in ((102, args.occupancy if args.occupancy else -1), (bre.OPT_TILE_LEAF, args.tile_leaf or -1),
                     (107, args.block_map), (105, args.sort_key), (108, args.tscan), (110, args.beam_key),
                     (111, args.margin), (112, args.tile_axis), (113, args.split_records), (114, args.film_compose),
                     (116, args.photon_single), (117, args.pass_priority),
                     (109, args.partial_mib), (118, args.readback), (119, args.slot_passes),
                     (121, args.coarse_keys)):
        if val >= 0:
            c.set_option(opt, val)
    if film_classes(args) > 1:
        c.set_film_classes(bre.FILM_CLASSES)
    st = torch.cuda.Stream(dev, priority=priority)
    c.set_stream(st.cuda_stream)
    return c, st


def counter_block(st, args):
    """libbre's counters of one gather (counting instantiation) as per-estimate / per-wave figures."""
    nseg_d = max(st["n_segments"], 1)
    items = (nseg_d + 63) // 64 * args.split  # (packet, subtree) work items = waves
    return {
        "candidates_per_estimate": st["candidates"] / nseg_d,
        "contributions_per_estimate": st["contributions"] / nseg_d,
        "node_visits_per_wave": st["node_visits"] / items,
        "leaf_visits_per_wave": st["leaf_visits"] / items,
        "beam_lines_staged_per_wave": st["beam_evals"] / items,
        "exact_batches_per_wave": st["ccp_wave_evals"] / items,
        "bundle_keep_frac": st["useful_beam_evals"] / max(st["beam_evals"], 1),
        "queued_pairs_per_estimate": st["queued_pairs"] / nseg_d,
        "contributions_per_queued_pair": st["contributions"] / max(st["queued_pairs"], 1),
        # (lane, kept beam) prefilter tests ~ kept beams x 64 lanes; per queued pair (~7)
        "prefilter_tests_per_queued_pair": st["useful_beam_evals"] * 64 / max(st["queued_pairs"], 1),
    }


def roofline(st, args, wl, gather_ms, pmc, cpu):
    """Roofline of the tile kernel for one launch of iteration 0 (see the module docstring).

    The arithmetic roofline is VALU issue (`issue` also carries the TA / TD busy
    fractions of the vector-memory path, the busiest unit since round 3): `achieved` = the launch's wave64 VALU instructions
    (SQ_INSTS_VALU) per second, `peak` = 256 CU x 4 SIMD x one wave64 instruction per 2 clocks at the
    clock the same counters measured, so `frac` = the VALU issue fraction.  The byte side is kept in
    `hbm`: the bytes the packets request per launch against the 8 TB/s HBM peak (served
    mostly from L1 / L2 / Infinity Cache: the requests exceed what HBM could deliver) and the HBM
    traffic the FETCH/WRITE counters measure.  Without the PMC passes the line falls back to the HBM
    roofline of the requested bytes."""
    nseg = max(st["n_segments"], 1)
    items = (nseg + 63) // 64 * args.split
    # what the packet algorithm requests from the memory hierarchy per launch (L1 / TA level): every
    # visited node record (the 4-wide walk's 128-B Node4; node_visits counts its visits) and staged beam
    # line (64 B) of every (packet, subtree) item; per item the
    # segments (40 B in) and the per-subtree partial sums (12 B out) of its 64 lanes; per queued
    # (lane, beam) pair the exact stage's loads (three of the segment's 16-B SegRec planes -- the unit
    # direction is recomputed -- and the 64-B BeamRec, which carries the power of the photon pass's
    # uniform-radius beams: 112 B; 128 B with the split layout, option 113); and the reduce (12 B x
    # split in, 12 B out per segment)
    queued = st.get("queued_pairs", 0)
    pair_b = 128.0 if args.split_records == 1 else 112.0
    req = (NODE4_BYTES * st["node_visits"] + 64.0 * st["beam_evals"] + items * 64 * (40 + 12) + pair_b * queued
           + nseg * 12 * (args.split + 1))
    requested = req / (gather_ms * 1e-3) / 1e9
    hbm = {"requested_GBps": requested, "peak": HBM_PEAK_GBPS, "requested_over_peak": requested / HBM_PEAK_GBPS,
           "requested_bytes_per_launch": req, "queued_pairs_per_launch": queued,
           "requested_model": "bytes the packets request at the L1 / texture-address level: 128 B x node "
                              "visits (4-wide Node4 records) + 64 B x beam lines staged + 52 B x 64 per (packet, "
                              "subtree) item + "
                              f"{pair_b:.0f} B per queued exact-stage pair + 12 B x (split + 1) per segment; counts "
                              "from this run's counter pass.  Served mostly by L1 / L2 / Infinity Cache: compare "
                              "traffic_bytes_per_launch (HBM) and the l2 block"}
    out = {"bound": "hbm", "achieved": requested, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
           "frac": requested / HBM_PEAK_GBPS, "traffic": None,
           "kernel": "k_gather_tile (+ k_reduce)", "launch": "iteration 0", "launch_ms": gather_ms}
    if pmc:
        out["traffic"] = pmc.get("traffic_bytes_per_launch")
        out["traffic_source"] = pmc.get("source")
        if out["traffic"]:
            hbm["traffic_bytes_per_launch"] = out["traffic"]
            hbm["traffic_GBps"] = out["traffic"] / (pmc["kernel_ms"] * 1e-3) / 1e9
            hbm["traffic_frac"] = hbm["traffic_GBps"] / HBM_PEAK_GBPS
            hbm["traffic_over_requested"] = out["traffic"] / req
        if pmc.get("l2"):
            out["l2"] = pmc["l2"]
        iss = pmc.get("issue")
        if iss:
            t = pmc["kernel_ms"] * 1e-3
            clock_hz = iss["clocks"] / t
            out.update({"bound": "valu_issue", "unit": "G wave64 VALU inst/s",
                        "achieved": iss["SQ_INSTS_VALU"] / t / 1e9,
                        "peak": CUS * SIMDS / 2.0 * clock_hz / 1e9,
                        "frac": iss["valu_issue_frac"], "clock_GHz": clock_hz / 1e9,
                        "pmc_launch_ms": pmc["kernel_ms"]})
            out["issue"] = iss
    out["hbm"] = hbm
    if cpu and cpu.get("visit_mean"):
        # SURVEY.md §8d's reference-tree model (every segment streams its candidates from HBM):
        # kept for comparison, not a fraction of HBM peak
        bpe = 32 + 12 + 32 * cpu["visit_mean"] + 40 * cpu["cand_mean"]
        out["ref_model_bytes_per_estimate"] = bpe
        out["ref_model_GBps"] = bpe * wl.segments_per_gather() / (gather_ms * 1e-3) / 1e9
        out["ref_model_V_C"] = [cpu["visit_mean"], cpu["cand_mean"]]
    return out


PMC_PASSES = {
    "fetch": ["FETCH_SIZE"],
    "write": ["WRITE_SIZE"],
    "sq": ["SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_INSTS_VALU", "SQ_INSTS_LDS",
           "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS", "SQ_LDS_IDX_ACTIVE", "GRBM_GUI_ACTIVE"],
    # the vector-memory path: address (TA) and data-return (TD) units, one each per CU
    "vmem": ["TA_TA_BUSY_sum", "TD_TD_BUSY_sum", "SQ_INSTS_VMEM_RD"],
    # where the requests are served: L2 hits / misses and the L1 -> L2 read requests (optional pass)
    "l2": ["TCC_HIT_sum", "TCC_MISS_sum", "TCP_TCC_READ_REQ_sum"],
}
PMC_OPTIONAL = {"l2"}


def pmc_passes(args):
    """This run's own rocprofv3 PMC passes (one counter group per pass, MI355X_MICROARCH.md
    §rocprofv3): a child process runs one untimed iteration of the same workload per pass.  Returns
    per-launch HBM bytes and the SQ issue figures of the tile kernel, or None if rocprofv3 is absent
    or a pass fails (the bench line then has traffic null)."""
    import csv
    import shutil

    prof = shutil.which("rocprofv3") or ("/opt/rocm/bin/rocprofv3" if os.path.exists("/opt/rocm/bin/rocprofv3") else None)
    if not prof:
        return None
    child = [sys.executable, os.path.abspath(__file__), "--pmc-child", "--workload", args.workload, "--steps", "1",
             "--warmup", "0", "--photons", str(args.photons), "--width", str(args.width), "--height",
             str(args.height), "--kernel", str(args.kernel), "--split", str(args.split), "--radius", str(args.radius)]
    vals, durs = {}, []
    tmp = tempfile.mkdtemp(prefix="bre_pmc_")
    env = dict(os.environ, TMPDIR="/tmp")
    for name, ctrs in PMC_PASSES.items():
        d = os.path.join(tmp, name)
        cmd = [prof, "--pmc", *ctrs, "--kernel-trace", "--output-format", "csv", "-d", d, "-o", "run", "--", *child]
        try:
            r = subprocess.run(cmd, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=150)
        except subprocess.TimeoutExpired:
            if name in PMC_OPTIONAL:
                continue
            return None
        if r.returncode != 0:
            if name in PMC_OPTIONAL:
                continue
            return None
        cc = kt = None
        for root_, _, files in os.walk(d):
            for f in files:
                if f.endswith("counter_collection.csv"):
                    cc = os.path.join(root_, f)
                if f.endswith("kernel_trace.csv"):
                    kt = os.path.join(root_, f)
        if not cc:
            if name in PMC_OPTIONAL:
                continue
            return None
        for row in csv.DictReader(open(cc)):
            if "k_gather_tile" in row["Kernel_Name"]:
                vals[row["Counter_Name"]] = vals.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
        if kt and not durs:
            for row in csv.DictReader(open(kt)):
                if "k_gather_tile" in row["Kernel_Name"]:
                    durs.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6)
    shutil.rmtree(tmp, ignore_errors=True)
    if not durs or "FETCH_SIZE" not in vals:
        return None
    # FETCH_SIZE / WRITE_SIZE in KB; gfx950 FETCH_SIZE reads half the bytes of wide streaming reads
    traffic = vals["FETCH_SIZE"] * 1024 * 2 + vals.get("WRITE_SIZE", 0.0) * 1024
    res = {"traffic_bytes_per_launch": traffic, "kernel_ms": float(np.mean(durs)),
           "source": "this run's rocprofv3 --pmc passes (1 iteration, iteration 0: the largest radius)"}
    clocks = vals.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
    if clocks > 0 and vals.get("SQ_WAVE_CYCLES"):
        wc = vals["SQ_WAVE_CYCLES"]
        res["issue"] = {
            "valu_issue_frac": vals["SQ_INSTS_VALU"] / (CUS * SIMDS / 2.0 * clocks),
            "lds_busy_frac": vals.get("SQ_LDS_IDX_ACTIVE", 0.0) / (CUS * clocks),
            "wait_any_frac": vals.get("SQ_WAIT_ANY", 0.0) / wc,
            "wait_inst_any_frac": vals.get("SQ_WAIT_INST_ANY", 0.0) / wc,
            "wait_inst_lds_frac": vals.get("SQ_WAIT_INST_LDS", 0.0) / wc,
            "valu_active_frac_of_wave_cycles": vals.get("SQ_ACTIVE_INST_VALU", 0.0) / wc,
            "SQ_INSTS_VALU": vals["SQ_INSTS_VALU"], "SQ_INSTS_LDS": vals.get("SQ_INSTS_LDS"),
            "clocks": clocks,
            "model": "VALU peak = 256 CU x 4 SIMD-32 / 2 clocks per wave64 instruction; LDS busy = "
                     "SQ_LDS_IDX_ACTIVE / (256 x clocks); TA / TD busy = TA_TA_BUSY_sum / TD_TD_BUSY_sum "
                     "/ (256 x clocks); clocks = GRBM_GUI_ACTIVE / 8 XCDs",
        }
        if "TD_TD_BUSY_sum" in vals:
            iss = res["issue"]
            iss["ta_busy_frac"] = vals.get("TA_TA_BUSY_sum", 0.0) / (CUS * clocks)
            iss["td_busy_frac"] = vals["TD_TD_BUSY_sum"] / (CUS * clocks)
            iss["SQ_INSTS_VMEM_RD"] = vals.get("SQ_INSTS_VMEM_RD")
            # the busiest of the kernel's units (the TD data-return path)
            units = {"valu_issue": iss["valu_issue_frac"], "lds": iss["lds_busy_frac"],
                     "vmem_address_ta": iss["ta_busy_frac"], "vmem_data_td": iss["td_busy_frac"]}
            iss["busiest_unit"] = max(units, key=units.get)
    if "TCC_HIT_sum" in vals and "TCC_MISS_sum" in vals:
        h, m = vals["TCC_HIT_sum"], vals["TCC_MISS_sum"]
        res["l2"] = {"TCC_HIT_sum": h, "TCC_MISS_sum": m, "hit_rate": h / max(h + m, 1.0),
                     "TCP_TCC_READ_REQ_sum": vals.get("TCP_TCC_READ_REQ_sum"),
                     "note": "L2 (TCC) requests of the iteration-0 launch: hits are served on the XCD, misses go "
                             "to the Infinity Cache / HBM (FETCH_SIZE); TCP_TCC_READ_REQ = L1 misses sent to L2"}
    return res


class SceneWorkload:
    """BASELINE.json configs[1..4] as full renders: c2 Cornell box + homogeneous fog (sigma_a 0.05,
    sigma_s 0.5, g 0); c3/c5 the same box filled with a 64^3 GridDensityMedium of seeded value-noise
    smoke (sigma_a 0.5, sigma_s 4.5, g 0.7); c4 the fog at 2048^2 with 20M photons."""

    def __init__(self, args, bre, ctxs, frame, shard_rank, shard_count):
        import torch

        sc = importlib.import_module("beam-radiance-estimate-pbrt_amd.scene")
        self.ctxs = ctxs  # [(BeamGather, torch stream)]: 1, or 2 when pipelined
        g = ctxs[0][0]
        self.args, self.bre, self.g, self.frame = args, bre, g, frame
        self.name = args.workload
        preset = WORKLOADS[args.workload]
        if preset["medium"] == "smoke":
            self.scene = sc.cornell_smoke_scene(0.5, 4.5, preset["g"], n=args.grid_n, seed=7)
        else:
            self.scene = sc.cornell_scene(0.05, 0.5, preset["g"])
        self.W, self.H = frame.w, frame.h
        for c, _ in ctxs:
            c.set_shard(shard_rank, shard_count, frame.block, frame.packets, roots=args.shard_mode == "roots")
        self.shard = (shard_rank, shard_count)
        self.ld = frame.accum
        # one iteration image per context (the camera pass's surface radiance, then the gather's
        # per-pixel sums, both deterministic: libbre adds a pixel's segments in depth order without
        # atomics), added to the ONE film in iteration order -- each add waits for the previous
        # iteration's add, whatever stream it ran on -- so the film's bits do not depend on the
        # number of contexts (tests/test_film_determinism_gpu.py)
        self.iter_img = [torch.zeros_like(self.ld) for _ in ctxs]
        self.scratch_film = torch.zeros_like(self.ld)
        self._last_add = None  # event after the previous iteration's film add
        self.data = (f"synthetic scene (SURVEY.md §8d {self.name.upper()}: built-in Cornell box + "
                     f"{'grid-density smoke' if preset['medium'] == 'smoke' else 'homogeneous fog'}; photons and "
                     "camera paths traced on the GPU)")
        self.last_nseg = 0
        self.n_iter = {"c2": 16, "c5": 10}.get(self.name)
        self._rec = {}
        if args.entry == "boundary":  # stage every timed iteration's recorder-order segments up front
            for k in range(max(args.steps, args.warmup)):
                self.recorder_segments(self.iteration(k))
            self.data += "; boundary leg: camera segments in recorder order through bre_gather_device"

    def radius(self, it):
        return self.bre.beam_radius_at(self.args.radius, self.args.alpha, it)

    def iteration(self, k):
        """Step k runs the render's iteration k mod its iteration count (C2: 16, C5: 10), so a longer
        --steps repeats the configuration's own iterations and never times smaller radii than it has."""
        return k % self.n_iter if self.n_iter else k

    def recorder_segments(self, it):
        """Boundary leg: iteration `it`'s camera segments in the reference's recorder order, on the
        device (untimed setup).  The camera pass of photonbeam.cpp:444-557 records per thread: 16x16
        tiles (:345-347) dealt by ParallelFor2D to the threads (here tile t to thread t mod 16), each
        tile's pixels row-major, each pixel's path depths in order; the recorders are concatenated in
        thread order (the mirror's Gather(recorders))."""
        import torch

        if it in self._rec:
            return self._rec[it]
        g = self.g
        g.camera_pass(self.scene, self.W, self.H, it, self.args.max_depth, True, True)
        s = g.get_segments()
        px = s["pixel"].astype(np.int64)
        x, y = px % self.W, px // self.W
        ntx = (self.W + 15) // 16
        tile = (y // 16) * ntx + x // 16
        key = ((((tile % 16) * (tile.max() + 1) + tile) * 256 + (y % 16) * 16 + x % 16) * 64 + s["depth"])
        order = np.argsort(key, kind="stable")
        dev = self.ld.device
        rec = {k: torch.from_numpy(np.ascontiguousarray(s[k][order])).to(dev) for k in ("o", "p", "d", "tmax", "pixel")}
        self._rec[it] = rec
        return rec

    def step(self, k, ev, scratch, ctx=None):
        import torch

        a = self.args
        it = self.iteration(k)
        i = k % len(self.ctxs) if ctx is None else ctx
        g, st = self.ctxs[i]
        ld = self.iter_img[i]
        film = self.scratch_film if scratch else self.ld
        R = self.radius(it)
        rec = self.recorder_segments(it) if a.entry == "boundary" else None
        with torch.cuda.stream(st):
            # ld is zero here: it starts zeroed and the film add below clears it (a framework zero_ / add_
            # would queue multi-wave kernels that wait behind the other context's gather; bre_film_add's
            # one-wave kernel runs beside it, bre_slot.hip)
            self.nbeams = g.trace_photons(self.scene, a.photons, it, a.max_depth, R)  # photon pass + BVH build
            if rec is None:
                n = g.camera_pass(self.scene, self.W, self.H, it, a.max_depth, True, True, surface=ld)
            else:
                n = int(rec["tmax"].shape[0])
            if ev is not None:  # libbre records them around the tile kernel itself (bre_set_gather_events)
                g.set_gather_events(*ev)
            if rec is None:
                g.gather_camera(R, ld)  # asynchronous: the next step's passes overlap it on the other stream
            else:  # the C-ABI boundary: caller-order device segments, sorted and gathered inside libbre
                g.gather_device(rec["o"], rec["p"], rec["d"], rec["tmax"], rec["pixel"], R, self.W * self.H, accum=ld)
            if ev is not None:
                g.set_gather_events(None, None)
            if self._last_add is not None:
                st.wait_event(self._last_add)
            g.film_add(ld, film, clear_src=True)  # film += ld; ld = 0
            self._last_add = torch.cuda.Event()
            self._last_add.record(st)
        if self.args.shard_mode == "roots" and self.shard[1] > 1:  # every segment, 1/count of the subtrees
            r, cnt = self.shard
            n = n // cnt + (1 if r < n % cnt else 0)  # the ranks' shares sum to the estimates
        elif self.frame.packets and self.shard[1] > 1:  # this rank gathers its range of the packets
            n = self.bre.shard_segments(n, *self.shard, self.frame.block)
        self.last_nseg = n
        return n

    def finish(self):
        """The film is complete once the last iteration's add is: the first context's stream waits for
        it (the frame's collective runs on the current stream after this)."""
        import torch

        if self._last_add is not None:
            torch.cuda.current_stream().wait_event(self._last_add)

    def close(self):
        for c, _ in self.ctxs:  # unlink the pipelined contexts (bre_set_gather_after) before any is destroyed
            if getattr(c, "_after", None) is not None:
                c.set_gather_after(None)
        for c, _ in self.ctxs[1:]:
            c.close()

    def diagnostics(self, k=0):
        import torch

        self.step(k, None, scratch=True, ctx=0)  # the first context: the one with the counters on
        self.g.synchronize()
        torch.cuda.synchronize()
        st = self.g.stats()
        return {"beams_per_iteration": st["n_beams"], "photon_pass_ms": st["photon_ms"], "bvh_build_ms": st["build_ms"],
                "camera_pass_ms": st["camera_ms"], "gather_ms_iter0": st["gather_ms"]}

    def segments_per_gather(self):
        return self.last_nseg

    def cpu_inputs(self, it):
        """Beams and camera segments of iteration `it` (GPU-traced: bit-exact with the oracle's
        photon and camera passes, tests/test_photon_gpu.py, tests/test_camera_gpu.py)."""
        R = self.radius(it)
        self.g.trace_photons(self.scene, self.args.photons, it, self.args.max_depth, R)
        beams = self.g.get_beams()
        self.g.camera_pass(self.scene, self.W, self.H, it, self.args.max_depth, True, True)
        s = self.g.get_segments()
        return beams, {k: s[k] for k in ("o", "p", "d", "tmax", "pixel")}, R

    def config(self, world):
        a = self.args
        med = ("homogeneous fog (sigma_a 0.05, sigma_s 0.5, g 0)" if WORKLOADS[self.name]["medium"] == "fog" else
               f"GridDensityMedium smoke {a.grid_n}^3 (sigma_a 0.5, sigma_s 4.5, g 0.7)")
        film = (f"{a.width}x{a.height} per GPU" if a.scaling != "strong" else
                f"{a.width}x{a.height}, the sorted segment packets split over the GPUs" if a.shard_mode == "packets"
                else f"{a.width}x{a.height}, the BVH work roots split over the GPUs" if a.shard_mode == "roots"
                else f"{a.width}x{a.height} split by 16x16 tiles over the GPUs")
        return {"workload": f"{self.name.upper()}: Cornell box + {med}, {a.photons / 1e6:g}M photons/iteration, "
                            f"{film}, maxdepth {a.max_depth}, R0 {a.radius}, alpha {a.alpha}",
                "photons_per_iteration": a.photons, "image": [self.W, self.H], "iterations_timed": a.steps,
                "render_iterations": self.n_iter, "entry": ("bre_gather_camera" if a.entry == "camera" else
                                                            "bre_gather_device, recorder-order segments"),
                "parallelism": (f"segment packets x{world} ({a.scaling} scaling), photons traced and camera pass "
                                "on every rank, one RCCL gather of the ranks' packet-class film planes per written "
                                "image (the 1-GPU film bit for bit)"
                                if a.shard_mode == "packets" and film_classes(a) > 1 else
                                f"segment packets x{world} ({a.scaling} scaling), photons traced and camera pass "
                                "on every rank, one RCCL reduce of the partial films per written image"
                                if a.shard_mode == "packets" else
                                f"BVH work roots x{world} ({a.scaling} scaling), photons traced and camera pass "
                                "on every rank, one RCCL reduce of the partial films per written image"
                                if a.shard_mode == "roots" else
                                f"image tiles x{world} ({a.scaling} scaling), photons traced on every rank, "
                                "one RCCL gather of the owned-pixel bands per written image"),
                "kernel": KERNEL_NAMES.get(a.kernel, str(a.kernel)), "split": a.split,
                "prefilter": bool(a.prefilter), "sort_segments": bool(a.sort_segments)}


class SyntheticWorkload:
    """SURVEY.md §8d synthetic-fog: fixed beam set + one camera segment per pixel (kernel only)."""

    name = "synthetic"

    def __init__(self, args, bre, g, frame, dev):
        import torch

        synth = importlib.import_module("beam-radiance-estimate-pbrt_amd.synth")
        self.args, self.g, self.frame = args, g, frame
        self.beams = synth.fog_beams(args.beams, seed=12345, radius=args.radius)
        pixels = frame.pixels
        if args.segment_kind == "camera":
            self.segs = synth.camera_segments(frame.w, frame.h, seed=777, pixels=pixels)
        else:  # incoherent secondary segments, one per owned pixel
            self.segs = synth.bounce_segments(len(pixels), seed=778)
            self.segs["pixel"] = pixels.astype(np.int32)
        self.nseg = int(self.segs["tmax"].shape[0])
        self.dB = {k: torch.from_numpy(v).to(dev).contiguous() for k, v in self.beams.items()}
        self.dS = {k: torch.from_numpy(v).to(dev).contiguous() for k, v in self.segs.items()}
        self.scratch = torch.zeros_like(frame.accum)
        self.data = "synthetic (synthetic-fog: PCG32 seeds 12345 beams / 777 segments)"

    def step(self, it, ev, scratch):
        g, dB, dS = self.g, self.dB, self.dS
        acc = self.scratch if scratch else self.frame.accum
        g.set_beams_device(dB["start"], dB["end"], dB["radius"], dB["power"])
        if ev is not None:  # around the tile kernel (bre_set_gather_events)
            g.set_gather_events(*ev)
        g.gather_device(dS["o"], dS["p"], dS["d"], dS["tmax"], dS["pixel"], self.args.radius, self.frame.npix,
                        accum=acc)
        if ev is not None:
            g.set_gather_events(None, None)
        return self.nseg

    def diagnostics(self, k=0):
        self.step(0, None, scratch=True)
        self.g.synchronize()
        st = self.g.stats()
        return {"bvh_build_ms": st["build_ms"], "beams": st["n_beams"]}

    def segments_per_gather(self):
        return self.nseg

    def finish(self):
        pass

    def close(self):
        pass

    def cpu_inputs(self, it):
        return self.beams, self.segs, self.args.radius

    def config(self, world):
        a = self.args
        return {"workload": "synthetic-fog: 1M-photon beam set, one camera segment per pixel, R=0.01",
                "beams": a.beams, "segments_per_gpu": self.nseg, "image": [self.frame.w, self.frame.h],
                "parallelism": f"image tiles x{world}, beams replicated", "kernel": KERNEL_NAMES.get(a.kernel),
                "split": a.split, "prefilter": bool(a.prefilter)}


def host_threads():
    """The host threads this process may really use: its CPU affinity, capped by a cgroup CPU quota
    (a GPU box's share of a large host: affinity can list every CPU of the machine while the quota
    allows ~16), and by OMP_NUM_THREADS when that is set (the box sets it to its share)."""
    n = len(os.sched_getaffinity(0))
    notes = [f"affinity {n}"]
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(float(q) / float(per)))
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = max(1, q // per)
        except (OSError, ValueError):
            pass
    if quota:
        notes.append(f"cgroup quota {quota}")
        n = min(n, quota)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        notes.append(f"OMP_NUM_THREADS {omp}")
        n = min(n, int(omp))
    return n, ", ".join(notes)


def cpu_baseline(wl, args, gather_per_step):
    """Oracle = CPU restatement of the reference algorithm (not pbrt itself: the reference build was
    denied).  For iteration 0 and the smallest-radius timed iteration: the SAH build single-threaded
    (as photonbeambvh.cpp:232), then the gather of a random sample of that iteration's segments on
    every host thread this process may use (256-segment chunks pulled dynamically, like
    ParallelFor2D, parallel.cpp:247-299) and on 1 thread.  value = 1 / the mean over the sampled
    iterations of the seconds per estimate (all threads)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import load_oracle

    ora = load_oracle()
    threads, cpu_note = host_threads()
    iters = sorted({0, wl.iteration(late_step(wl, args.steps))}) if wl.name != "synthetic" else [0]
    per_it, visit, cand = [], [], []
    for it in iters:
        beams, segs, R = wl.cpu_inputs(it)
        t = time.perf_counter()
        bvh = ora.build(beams)
        build_s = time.perf_counter() - t
        n = segs["tmax"].shape[0]
        perm = np.random.default_rng(2024 + it).permutation(n)

        def take(idx):
            return {k: np.ascontiguousarray(v[idx]) for k, v in segs.items()}

        def timed(m, nthreads, off=0):
            smp = take(perm[off:off + m])
            t = time.perf_counter()
            out = bvh.gather(smp, R, nthreads=nthreads, chunk=max(1, min(256, m // (4 * nthreads) or 1)))
            return time.perf_counter() - t, out

        # calibrate, then size the samples: target_s / len(iters) on all threads, a quarter of that on 1
        dt, _ = timed(4 * threads, threads)
        per_seg = max(dt, 1e-3) / (4 * threads)
        tgt = args.cpu_seconds / len(iters)
        m = int(min(n, max(8 * threads, tgt / per_seg)))
        g_s, out = timed(m, threads)
        dt1, _ = timed(2, 1, off=m)
        m1 = int(min(n - m - 2, max(4, 0.5 * tgt / max(dt1 / 2, 1e-3))))
        g1_s, _ = timed(m1, 1, off=m + 2)
        bvh.close()
        nb = beams["radius"].shape[0]
        rec = {"iteration": it, "beams": nb, "sah_build_s": build_s, "segments_all_threads": m,
               "gather_all_threads_s": g_s, "estimates_per_s_all_threads": m / g_s, "segments_1_thread": m1,
               "gather_1_thread_s": g1_s, "estimates_per_s_1_thread": m1 / g1_s}
        if it < len(gather_per_step) and wl.segments_per_gather():
            rec["gpu_gather_only_estimates_per_s"] = wl.segments_per_gather() / (gather_per_step[it] * 1e-3)
        per_it.append(rec)
        visit.append(float(out["visit"].mean()))
        cand.append(float(out["cand"].mean()))
    value = 1.0 / float(np.mean([1.0 / r["estimates_per_s_all_threads"] for r in per_it]))
    value1 = 1.0 / float(np.mean([1.0 / r["estimates_per_s_1_thread"] for r in per_it]))
    return {
        "report": {
            "value": value,
            "unit": "estimates/s",
            "cores": threads,
            "nproc": os.cpu_count(),
            "kind": "port",
            "value_1_thread": value1,
            "threads_note": cpu_note,
            "sample": (f"random camera segments of the {wl.name} workload at iterations {iters} (the largest and "
                       f"smallest radius the line times), gathered against all of that iteration's beams through the oracle's SAH "
                       f"tree: {threads} threads (every CPU this process may use: {cpu_note}; nproc {os.cpu_count()}) "
                       f"and 1 thread; value = 1 / mean seconds per estimate over those iterations"),
            "per_iteration": per_it,
        },
        "visit_mean": float(np.mean(visit)),
        "cand_mean": float(np.mean(cand)),
    }


if __name__ == "__main__":
    main()
