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

`--workload synthetic` = SURVEY.md §8d synthetic-fog kernel-only set (1M beams, seed 12345; one
camera segment per pixel, seed 777): a step is BVH build + gather.

Multi-GPU (weak scaling): the film is 512 x (512*N); its 16x16 tiles (photonbeam.cpp:345-347) are
dealt round-robin to the N ranks; every rank traces the same photons (per-photon PCG32 sequences,
so no communication) and builds its own BVH; the framebuffer partial sums are reduced to rank 0
once per written image (the last step), one RCCL reduce.

Also reported: `roofline` (SURVEY.md §8d algorithmic bytes of the gather kernel vs HBM peak; the
gather kernel's average duration measured with HIP events on the stream it is launched on;
`traffic` = PMC FETCH_SIZE+WRITE_SIZE per launch from the committed rocprofv3 summary of the same
workload, when present) and `cpu_baseline` (the oracle's CPU restatement of the reference
algorithm — SAH tree, per-query vector<shared_ptr>, all host threads — timed on a bounded sample
of the same segments and beams; rank 0, N=1).
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
VALU_PEAK_TFLOPS = 157.3  # FP32 vector peak (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed iterations (default: c2 16 = the whole 16-spp render, c5 10 passes, else 4)")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=["c2", "c3", "c4", "c5", "synthetic"], default="c2",
                    help="BASELINE.json configs[1..4] (SURVEY.md §8d) or the kernel-only synthetic set")
    ap.add_argument("--photons", type=int, default=None, help="photons per iteration (c2 1M, c3 5M, c4 20M, c5 50M)")
    ap.add_argument("--beams", type=int, default=1_000_000, help="synthetic: beams")
    ap.add_argument("--width", type=int, default=None, help="film width (c2 512, c3/c5 1024, c4 2048)")
    ap.add_argument("--height", type=int, default=None, help="film height per GPU (weak) or total (strong)")
    ap.add_argument("--scaling", choices=["weak", "strong"], default=None,
                    help="weak: a W x (H*N) film, H rows per GPU (default); strong: one W x H film split by "
                         "16x16 tiles over the N GPUs (c4 default)")
    ap.add_argument("--grid-n", type=int, default=64, help="c3/c5: smoke density grid resolution")
    ap.add_argument("--radius", type=float, default=0.01, help="initialbeamradius (c2) / R (synthetic)")
    ap.add_argument("--alpha", type=float, default=0.5)
    ap.add_argument("--max-depth", type=int, default=5)
    ap.add_argument("--kernel", type=int, default=0)
    ap.add_argument("--leaf-size", type=int, default=1)
    ap.add_argument("--split", type=int, default=8, help="BVH subtrees per segment packet (kernels 1/3)")
    ap.add_argument("--prefilter", type=int, default=1)
    ap.add_argument("--chunk-len", type=int, default=400, help="kernel 5: chunk length in units of E/100")
    ap.add_argument("--chunk-leaf", type=int, default=1, help="kernel 5: chunks per LBVH leaf")
    ap.add_argument("--sort-segments", type=int, default=1, help="coherence-sort the camera segments (0/1)")
    ap.add_argument("--debug-mode", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--occupancy", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--loose-cos", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--tile-leaf", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--tile-mode", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--sort-key", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-diag", action="store_true", help="skip the untimed counters/timing pass (profiling runs)")
    ap.add_argument("--segment-kind", choices=["camera", "bounce"], default="camera",
                    help="synthetic: camera primary segments or incoherent bounce segments")
    ap.add_argument("--profile-summary", default=None,
                    help="rocprofv3 PMC summary (profiles/*/profile_summary.json) for roofline.traffic")
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    preset = WORKLOADS.get(a.workload, WORKLOADS["c2"])
    for k in ("steps", "photons", "width", "height", "scaling"):
        if getattr(a, k) is None:
            setattr(a, k, preset[k])
    return a


# BASELINE.json configs[1..4].  c4/c5 are 8-GPU configurations: at N=1 they run
# as stated (long) unless --photons / --width / --height scale them down.
WORKLOADS = {
    "c2": dict(steps=16, photons=1_000_000, width=512, height=512, scaling="weak", medium="fog", g=0.0),
    "c3": dict(steps=4, photons=5_000_000, width=1024, height=1024, scaling="weak", medium="smoke", g=0.7),
    "c4": dict(steps=4, photons=20_000_000, width=2048, height=2048, scaling="strong", medium="fog", g=0.0),
    "c5": dict(steps=10, photons=50_000_000, width=1024, height=1024, scaling="strong", medium="smoke", g=0.7),
    "synthetic": dict(steps=10, photons=0, width=512, height=512, scaling="weak", medium="fog", g=0.0),
}


# V (reference-tree node tests) and C (candidates) per estimate of each workload's iteration 0,
# measured by the oracle at N=1 (bench.py's CPU leg, profiles/r09/bench.json); used for the
# roofline fields when this run has no CPU leg.  The beams and segments do not depend on N.
ROOFLINE_REF = {
    "c2": {"V_ref_tree": 1365412.6795491143, "C": 420520.3309178744,
           "source": "profiles/r09/bench.json (oracle SAH tree, CPU sample of iteration 0)"},
}


KERNEL_NAMES = {0: "auto (kernel 4: leaf tiles of 64 beams, packet bundle reject, compacted pair queue)", 1: "depth-first wave-packet",
                2: "thread-per-segment", 3: "packet-proxy + depth-first hand-over",
                4: "leaf tiles + wavefront-compacted pair queue",
                5: "capsule-chunk index (contributing pairs only)",
                6: "hand-over (packet-proxy kernel 3 + leaf-tile kernel 4)"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    bre = importlib.import_module("beam-radiance-estimate-pbrt_amd")
    dmod = importlib.import_module("beam-radiance-estimate-pbrt_amd.dist")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if world > 1 else 0)

    W, H = args.width, args.height * (world if args.scaling == "weak" else 1)
    frame = dmod.ShardedFrame(W, H, rank, world, device=dev)
    g = bre.BeamGather(dev.index, kernel=args.kernel, leaf_size=args.leaf_size, split=args.split,
                       prefilter=bool(args.prefilter))
    g.set_option(bre.OPT_SORT_SEGMENTS, args.sort_segments)
    if args.kernel == 5:
        g.set_option(bre.OPT_CHUNK_LEN, args.chunk_len)
        g.set_option(bre.OPT_CHUNK_LEAF, args.chunk_leaf)
    if args.debug_mode:
        g.set_option(100, args.debug_mode)
    if args.occupancy:
        g.set_option(102, args.occupancy)
    if args.loose_cos:
        g.set_option(103, args.loose_cos)
    if args.tile_leaf:
        g.set_option(bre.OPT_TILE_LEAF, args.tile_leaf)
    if args.tile_mode >= 0:
        g.set_option(104, args.tile_mode)
    if args.sort_key >= 0:
        g.set_option(105, args.sort_key)
    # one explicit stream shared by libbre and torch: the HIP events that time the gather kernel
    # are recorded on the stream the kernel runs on
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    g.set_stream(stream.cuda_stream)

    if args.workload != "synthetic":
        wl = SceneWorkload(args, bre, g, frame, rank, world)
    else:
        wl = SyntheticWorkload(args, bre, g, frame, rank, world, dev)

    for k in range(args.warmup):
        wl.step(k, None, scratch=True)
    torch.cuda.synchronize(dev)

    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    nseg_local = 0
    for k in range(args.steps):
        nseg_local += wl.step(k, events[k], scratch=False)
        if k == args.steps - 1:
            frame.reduce_to_root(0)  # one RCCL reduce per written image (no-op at N=1)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    gather_ms = float(np.mean([a.elapsed_time(b) for a, b in events]))
    if world > 1:
        tt = torch.tensor([elapsed, gather_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, gather_ms = float(tt[0]), float(tt[1])
        tot = torch.tensor([nseg_local], dtype=torch.int64, device=dev)
        dist.all_reduce(tot)
        total_seg = int(tot.item())
    else:
        total_seg = nseg_local
    value = total_seg / elapsed

    # untimed: one more step with counters and per-phase HIP-event timing inside libbre
    if not args.no_diag:
        g.set_option(bre.OPT_COUNTERS, 1)
        g.set_option(bre.OPT_TIMING, 1)
        diag = wl.diagnostics()
    else:
        diag = {}
    st = g.stats()
    nseg_d = max(st["n_segments"], 1)
    waves = (nseg_d + 63) // 64
    c_mean = st["candidates"] / nseg_d

    result = {
        "metric": ("beam-radiance estimates/sec at 1M photons" if args.workload in ("c2", "synthetic") else
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
        "config": wl.config(),
        "estimates_per_step_per_gpu": nseg_local / args.steps,
        "gather_kernel_ms": gather_ms,
        "candidates_per_estimate": c_mean,
        "contributions_per_estimate": st["contributions"] / nseg_d,
        "candidate_pair_tests_per_s": c_mean * value,
        "node_visits_per_wave": st["node_visits"] / waves,
        "leaf_visits_per_wave": st["leaf_visits"] / waves,
        "beam_evals_per_wave": st["beam_evals"] / waves,
        "ccp_wave_evals_per_wave": st["ccp_wave_evals"] / waves,
        "max_stack_depth": st["max_stack_depth"],
        "redo_items": st["redo_items"],
        "prefilter_rejects_per_estimate": st["prefilter_rejects"] / nseg_d,
        "bundle_keep_frac": st["useful_beam_evals"] / max(st["beam_evals"], 1),
        "chunks": st.get("n_chunks", 0),
    }
    result.update(diag)

    def roofline(v_ref, c_ref, source):
        # SURVEY.md §8d algorithmic bytes per estimate: 32 + 12 + 32*V + 40*C, V and C from the
        # reference SAH tree (oracle) on a CPU sample of the same workload
        bytes_per_est = 32 + 12 + 32 * v_ref + 40 * c_ref
        per_launch = bytes_per_est * wl.segments_per_gather()
        achieved = per_launch / (gather_ms * 1e-3) / 1e9
        traffic = pmc_traffic(args.profile_summary or wl.default_profile())
        return {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBPS,
            "traffic": traffic,
            # the PMC-measured bytes per launch over this run's launch time: the HBM/fabric
            # bandwidth the kernel actually draws (the profile's launches average the same command)
            "traffic_GBps": traffic / (gather_ms * 1e-3) / 1e9 if traffic else None,
            "traffic_frac": traffic / (gather_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS if traffic else None,
            "algorithmic_bytes_per_launch": per_launch,
            "bytes_per_estimate": bytes_per_est,
            "V_ref_tree": v_ref,
            "C": c_ref,
            "V_C_source": source,
            "kernel": "gather (k_gather_tile; k_gather_proxy too in hand-over mode)",
        }

    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(wl.cpu_beams(), wl.cpu_segments(), wl.cpu_radius(), args.cpu_seconds, wl.name)
        result["cpu_baseline"] = cpu["report"]
        result["roofline"] = roofline(cpu["visit_mean"], cpu["cand_mean"], "oracle SAH tree on this run's CPU sample")
        result["speedup_vs_cpu"] = value / cpu["report"]["value"]
    elif rank == 0:
        # no CPU leg (N > 1, or --no-cpu): V and C of the same workload from the committed N=1 run
        ref = ROOFLINE_REF.get(args.workload) if (args.photons, args.width) == (
            WORKLOADS[args.workload]["photons"], WORKLOADS[args.workload]["width"]) else None
        if ref:
            result["roofline"] = roofline(ref["V_ref_tree"], ref["C"], ref["source"])
    g.close()
    if rank == 0:
        line = json.dumps(result)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.destroy_process_group()


def pmc_traffic(path):
    """HBM bytes per gather launch from a committed rocprofv3 PMC summary (FETCH_SIZE with the
    gfx950 correction + WRITE_SIZE, MI355X_MICROARCH.md), or None when absent."""
    if not path or not os.path.exists(path):
        return None
    with open(path) as f:
        summ = json.load(f)
    tot = 0.0
    calls = 0
    for name, v in summ.items():
        if name.startswith("k_gather"):
            if "hbm_read_bytes_corrected" not in v:
                continue
            tot += (v["hbm_read_bytes_corrected"] + v.get("hbm_write_bytes", 0.0)) * v["calls"]
            calls = max(calls, v["calls"])  # every gather launches each of its kernels once
    return tot / calls if calls else None


class SceneWorkload:
    """BASELINE.json configs[1..4] as full renders: c2 Cornell box + homogeneous fog (sigma_a 0.05,
    sigma_s 0.5, g 0); c3/c5 the same box filled with a 64^3 GridDensityMedium of seeded value-noise
    smoke (sigma_a 0.5, sigma_s 4.5, g 0.7); c4 the fog at 2048^2 with 20M photons."""

    def __init__(self, args, bre, g, frame, rank, world):
        import torch

        sc = importlib.import_module("beam-radiance-estimate-pbrt_amd.scene")
        self.args, self.bre, self.g, self.frame = args, bre, g, frame
        self.name = args.workload
        preset = WORKLOADS[args.workload]
        if preset["medium"] == "smoke":
            self.scene = sc.cornell_smoke_scene(0.5, 4.5, preset["g"], n=args.grid_n, seed=7)
        else:
            self.scene = sc.cornell_scene(0.05, 0.5, preset["g"])
        self.W, self.H = frame.w, frame.h
        g.set_shard(rank, world)
        self.ld = frame.accum
        self.scratch = torch.zeros_like(self.ld)
        self.world = world
        self.data = (f"synthetic scene (SURVEY.md §8d {self.name.upper()}: built-in Cornell box + "
                     f"{'grid-density smoke' if preset['medium'] == 'smoke' else 'homogeneous fog'}; photons and "
                     "camera paths traced on the GPU)")
        self.last_nseg = 0

    def radius(self, it):
        return self.bre.beam_radius_at(self.args.radius, self.args.alpha, it)

    def step(self, it, ev, scratch):
        a, g = self.args, self.g
        ld = self.scratch if scratch else self.ld
        R = self.radius(it)
        self.nbeams = g.trace_photons(self.scene, a.photons, it, a.max_depth, R)  # photon pass + BVH build
        n = g.camera_pass(self.scene, self.W, self.H, it, a.max_depth, True, True, surface=ld)
        if ev is not None:
            ev[0].record()
        g.gather_camera(R, ld)
        if ev is not None:
            ev[1].record()
        self.last_nseg = n
        return n

    def diagnostics(self):
        import torch

        it = 0
        self.step(it, None, scratch=True)
        self.g.synchronize()
        torch.cuda.synchronize()
        st = self.g.stats()
        self.R0 = self.radius(it)
        return {"beams_per_iteration": st["n_beams"], "photon_pass_ms": st["photon_ms"], "bvh_build_ms": st["build_ms"],
                "camera_pass_ms": st["camera_ms"], "gather_ms_iter0": st["gather_ms"]}

    def segments_per_gather(self):
        return self.last_nseg

    def cpu_beams(self):
        self.g.trace_photons(self.scene, self.args.photons, 0, self.args.max_depth, self.radius(0))
        return self.g.get_beams()

    def cpu_segments(self):
        self.g.camera_pass(self.scene, self.W, self.H, 0, self.args.max_depth, True, True)
        s = self.g.get_segments()
        return {k: s[k] for k in ("o", "p", "d", "tmax", "pixel")}

    def cpu_radius(self):
        return self.radius(0)

    def default_profile(self):
        if self.name != "c2":
            return None
        return os.path.join(ROOT, "profiles", "r09", "profile_summary.json")

    def config(self):
        a = self.args
        med = ("homogeneous fog (sigma_a 0.05, sigma_s 0.5, g 0)" if WORKLOADS[self.name]["medium"] == "fog" else
               f"GridDensityMedium smoke {a.grid_n}^3 (sigma_a 0.5, sigma_s 4.5, g 0.7)")
        film = f"{a.width}x{a.height} per GPU" if a.scaling == "weak" else f"{a.width}x{a.height} split over the GPUs"
        return {"workload": f"{self.name.upper()}: Cornell box + {med}, {a.photons / 1e6:g}M photons/iteration, "
                            f"{film}, maxdepth {a.max_depth}, R0 {a.radius}, alpha {a.alpha}",
                "photons_per_iteration": a.photons, "image": [self.W, self.H], "iterations_timed": a.steps,
                "parallelism": f"image-tiles x{self.world}, photons traced on every rank",
                "kernel": KERNEL_NAMES[a.kernel], "leaf_size": a.leaf_size, "split": a.split,
                "prefilter": bool(a.prefilter), "sort_segments": bool(a.sort_segments)}


class SyntheticWorkload:
    """SURVEY.md §8d synthetic-fog: fixed beam set + one camera segment per pixel (kernel only)."""

    name = "synthetic"

    def __init__(self, args, bre, g, frame, rank, world, dev):
        import torch

        synth = importlib.import_module("beam-radiance-estimate-pbrt_amd.synth")
        self.args, self.g, self.frame, self.world = args, g, frame, world
        self.beams = synth.fog_beams(args.beams, seed=12345, radius=args.radius)
        pixels = frame.pixels
        if args.segment_kind == "camera":
            self.segs = synth.camera_segments(frame.w, frame.h, seed=777, pixels=pixels)
        else:  # incoherent secondary segments, one per owned pixel
            self.segs = synth.bounce_segments(len(pixels), seed=778 + rank)
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
        if ev is not None:
            ev[0].record()
        g.gather_device(dS["o"], dS["p"], dS["d"], dS["tmax"], dS["pixel"], self.args.radius, self.frame.npix,
                        accum=acc)
        if ev is not None:
            ev[1].record()
        return self.nseg

    def diagnostics(self):
        self.step(0, None, scratch=True)
        self.g.synchronize()
        st = self.g.stats()
        return {"bvh_build_ms": st["build_ms"], "beams": st["n_beams"]}

    def segments_per_gather(self):
        return self.nseg

    def cpu_beams(self):
        return self.beams

    def cpu_segments(self):
        return self.segs

    def cpu_radius(self):
        return self.args.radius

    def default_profile(self):
        return os.path.join(ROOT, "profiles", "r02", "profile_summary.json")

    def config(self):
        a = self.args
        return {"workload": "C2 synthetic-fog: 1M-photon beam set, 512x512 camera segments per GPU, R=0.01",
                "beams": a.beams, "segments_per_gpu": self.nseg, "image": [self.frame.w, self.frame.h],
                "parallelism": f"image-tiles x{self.world}, beams replicated", "kernel": KERNEL_NAMES[a.kernel],
                "leaf_size": a.leaf_size, "split": a.split, "prefilter": bool(a.prefilter)}


def cpu_baseline(beams, segs, R, target_s, name):
    """Oracle = CPU restatement of the reference algorithm (not pbrt itself: the reference build was
    denied).  SAH build single-threaded (as photonbeambvh.cpp:232), gather on all
    available host threads over 256-segment chunks pulled dynamically (ParallelFor2D-like)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import load_oracle

    ora = load_oracle()
    threads = max(1, min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))
    t = time.perf_counter()
    bvh = ora.build(beams)
    build_s = time.perf_counter() - t
    n = segs["tmax"].shape[0]
    rng = np.random.default_rng(2024)
    perm = rng.permutation(n)

    def take(idx):
        return {k: np.ascontiguousarray(v[idx]) for k, v in segs.items()}

    # calibrate on a small sample, then size the timed sample to ~target_s
    probe = take(perm[: 4 * threads])
    t = time.perf_counter()
    bvh.gather(probe, R, nthreads=threads, chunk=1)
    dt = max(time.perf_counter() - t, 1e-3)
    per_seg = dt / probe["tmax"].shape[0]
    m = int(min(n, max(8 * threads, target_s / per_seg)))
    sample = take(perm[:m])
    t = time.perf_counter()
    out = bvh.gather(sample, R, nthreads=threads, chunk=max(1, min(256, m // (4 * threads) or 1)))
    gather_s = time.perf_counter() - t
    bvh.close()
    nb = beams["radius"].shape[0]
    return {
        "report": {
            "value": m / gather_s,
            "unit": "estimates/s",
            "cores": threads,
            "kind": "port",
            "sample": f"{m} random camera segments of the {name} workload (iteration 0), gather {gather_s:.1f} s on "
                      f"{threads} threads against all {nb} beams; SAH build of the {nb} beams took {build_s:.1f} s "
                      f"(1 thread, not in value)",
            "sah_build_s": build_s,
        },
        "visit_mean": float(out["visit"].mean()),
        "cand_mean": float(out["cand"].mean()),
    }


if __name__ == "__main__":
    main()
