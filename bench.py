#!/usr/bin/env python3
"""Benchmark: beam-radiance estimates/sec at 1M photons (BASELINE.json metric), MI355X.

Workload (config C2 of BASELINE.json, synthetic-fog of SURVEY.md §8d): 1,000,000 photon beams
(radius 0.01, length ~ Exp(0.25) in the unit cube, PCG32 seed 12345) and one camera segment per
pixel of a 512x512 image per GPU (seed 777); R_cur = 0.01.  One *step* is one iteration of the
hot path with inputs already resident in HBM: the GPU BVH build over the iteration's beams
(replacing PhotonBeamBVH's ctor) + the gather over every camera segment (photonbeam.cpp:494-508)
accumulating into the framebuffer; with N>1 ranks, + one RCCL reduce of the framebuffer to rank 0.
One *estimate* = the full gather for one segment.  value = all ranks' segments * steps / max-rank
wall time of the timed steps.

Multi-GPU (weak scaling): the image is 512 x (512*N); its 16x16 tiles are dealt round-robin to the
N ranks (photonbeam.cpp:345-347 tiles); the beams are replicated (every rank regenerates them from
the same seeds) and each rank builds its own BVH; the framebuffer partial sums are reduced to rank 0.

Also reported: `roofline` (SURVEY.md §8d algorithmic bytes of the gather kernel vs HBM peak; the
kernel's average duration is measured with HIP events on the stream it is launched on) and
`cpu_baseline` (the oracle's CPU restatement of the reference algorithm — SAH tree, per-query
vector<shared_ptr>, all host threads — timed on a bounded sample of the same segments; rank 0, N=1).
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
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--beams", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--height", type=int, default=512)
    ap.add_argument("--radius", type=float, default=0.01)
    ap.add_argument("--kernel", type=int, default=0)
    ap.add_argument("--leaf-size", type=int, default=1)
    ap.add_argument("--split", type=int, default=16, help="BVH subtrees per segment packet (kernels 1/3)")
    ap.add_argument("--prefilter", type=int, default=1)
    ap.add_argument("--debug-mode", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--occupancy", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--segment-kind", choices=["camera", "bounce"], default="camera",
                    help="camera: C2 primary segments (default, the metric); bounce: incoherent segments")
    ap.add_argument("--json-out", default=None)
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    bre = importlib.import_module("beam-radiance-estimate-pbrt_amd")
    synth = importlib.import_module("beam-radiance-estimate-pbrt_amd.synth")
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

    W, H = args.width, args.height * world
    frame = dmod.ShardedFrame(W, H, rank, world, device=dev)
    npix = frame.npix
    pixels = frame.pixels
    beams = synth.fog_beams(args.beams, seed=12345, radius=args.radius)
    if args.segment_kind == "camera":
        segs = synth.camera_segments(W, H, seed=777, pixels=pixels)
    else:  # incoherent secondary segments, one per owned pixel
        segs = synth.bounce_segments(len(pixels), seed=778 + rank)
        segs["pixel"] = pixels.astype(np.int32)
    nseg = int(segs["tmax"].shape[0])
    dB = {k: torch.from_numpy(v).to(dev).contiguous() for k, v in beams.items()}
    dS = {k: torch.from_numpy(v).to(dev).contiguous() for k, v in segs.items()}
    accum = frame.accum

    g = bre.BeamGather(dev.index, kernel=args.kernel, leaf_size=args.leaf_size, split=args.split,
                       prefilter=bool(args.prefilter))
    if args.debug_mode:
        g.set_option(100, args.debug_mode)
    if args.occupancy:
        g.set_option(102, args.occupancy)
    # one explicit stream shared by libbre and torch: the HIP events that time the gather kernel
    # are recorded on the stream the kernel runs on
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    g.set_stream(stream.cuda_stream)
    R = args.radius

    def step(ev=None):
        g.set_beams_device(dB["start"], dB["end"], dB["radius"], dB["power"])
        if ev is not None:
            ev[0].record(stream)
        g.gather_device(dS["o"], dS["p"], dS["d"], dS["tmax"], dS["pixel"], R, npix, accum=accum)
        if ev is not None:
            ev[1].record(stream)
        frame.reduce_to_root(0)  # one RCCL reduce per written image (no-op at N=1)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)

    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(events[k])
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
        tot = torch.tensor([nseg], dtype=torch.int64, device=dev)
        dist.all_reduce(tot)
        total_seg = int(tot.item())
    else:
        total_seg = nseg

    # untimed: counters and build time (HIP events inside libbre, same stream)
    g.set_option(bre.OPT_COUNTERS, 1)
    g.set_option(bre.OPT_TIMING, 1)
    g.set_beams_device(dB["start"], dB["end"], dB["radius"], dB["power"])
    tmp = torch.zeros_like(accum)
    g.gather_device(dS["o"], dS["p"], dS["d"], dS["tmax"], dS["pixel"], R, npix, accum=tmp)
    g.synchronize()
    st = g.stats()
    g.close()

    value = total_seg * args.steps / elapsed
    c_mean = st["candidates"] / max(nseg, 1)
    contrib_mean = st["contributions"] / max(nseg, 1)
    waves = (nseg + 63) // 64

    result = {
        "metric": "beam-radiance estimates/sec at 1M photons",
        "value": value,
        "unit": "estimates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (synthetic-fog: PCG32 seeds 12345 beams / 777 segments)",
        "config": {
            "workload": "C2 synthetic-fog: 1M-photon beam set, 512x512 camera segments per GPU, R=0.01",
            "beams": args.beams,
            "segments_per_gpu": nseg,
            "image": [W, H],
            "parallelism": f"image-tiles x{world}, beams replicated",
            "kernel": {0: "auto (packet-proxy + depth-first hand-over)", 1: "depth-first wave-packet",
                       2: "thread-per-segment", 3: "packet-proxy + depth-first hand-over"}[args.kernel],
            "leaf_size": args.leaf_size,
            "split": args.split,
            "prefilter": bool(args.prefilter),
        },
        "gather_kernel_ms": gather_ms,
        "bvh_build_ms": st["build_ms"],
        "candidates_per_estimate": c_mean,
        "contributions_per_estimate": contrib_mean,
        "candidate_pair_tests_per_s": c_mean * value,
        "node_visits_per_wave": st["node_visits"] / max(waves, 1),
        "leaf_visits_per_wave": st["leaf_visits"] / max(waves, 1),
        "beam_evals_per_wave": st["beam_evals"] / max(waves, 1),
        "ccp_wave_evals_per_wave": st["ccp_wave_evals"] / max(waves, 1),
        "useful_beam_evals_per_wave": st["useful_beam_evals"] / max(waves, 1),
        "max_stack_depth": st["max_stack_depth"],
        "redo_items": st["redo_items"],
        "prefilter_rejects_per_estimate": st["prefilter_rejects"] / max(nseg, 1),
    }

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(beams, segs, R, args.cpu_seconds)
        result["cpu_baseline"] = cpu["report"]
        # SURVEY §8d algorithmic bytes per estimate: 32 + 12 + 32*V + 40*C, V and C from the
        # reference SAH tree (oracle) on the CPU sample
        v_ref, c_ref = cpu["visit_mean"], cpu["cand_mean"]
        bytes_per_est = 32 + 12 + 32 * v_ref + 40 * c_ref
        achieved = bytes_per_est * nseg / (gather_ms * 1e-3) / 1e9
        result["roofline"] = {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBPS,
            "traffic": None,
            "bytes_per_estimate": bytes_per_est,
            "V_ref_tree": v_ref,
            "C": c_ref,
        }
        result["speedup_vs_cpu"] = value / cpu["report"]["value"]
    if rank == 0:
        line = json.dumps(result)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(beams, segs, R, target_s):
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
    return {
        "report": {
            "value": m / gather_s,
            "unit": "estimates/s",
            "cores": threads,
            "kind": "port",
            "sample": f"{m} random camera segments of the same 512x512 workload, {gather_s:.1f} s gather on "
                      f"{threads} threads; SAH build of {beams['radius'].shape[0]} beams took {build_s:.1f} s "
                      f"(1 thread, not in value)",
            "sah_build_s": build_s,
        },
        "visit_mean": float(out["visit"].mean()),
        "cand_mean": float(out["cand"].mean()),
    }


if __name__ == "__main__":
    main()
