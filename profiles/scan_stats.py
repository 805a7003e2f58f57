"""Scan shape of the production tile kernel on real C2/C3 iterations, from a BRE_SCAN_STATS=1 build
(profiles/variant.sh scan "-DBRE_SCAN_STATS=1"):
    BRE_LIBRARY=.../libbre_scan.so python profiles/scan_stats.py [c2|c3] [iterations...]
Per leaf-tile visit: lanes on the tile, beams kept by the packet rejects, scan steps taken (beam-major
two beams per step, or one on-lane per step when transposed), min(on, kept), the steps a full
(lane, beam) pair compaction would take, queued pairs, and the fraction of transposed tiles."""
import importlib
import json
import sys

import os
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

bre = importlib.import_module("beam-radiance-estimate-pbrt_amd")
sc = importlib.import_module("beam-radiance-estimate-pbrt_amd.scene")
args = sys.argv[1:]
opts = [tuple(int(v) for v in a[4:].split("=")) for a in args if a.startswith("opt:")]  # opt:112=1
args = [a for a in args if not a.startswith("opt:")]
wl = "c2"
if args and args[0] in ("c2", "c3"):
    wl = args.pop(0)
its = [int(x) for x in args] or [0, 8]
# c2: Cornell fog, 1M photons, 512^2; c3: 64^3 smoke (bench.py's preset), 5M photons, 1024^2
if wl == "c3":
    scene = sc.cornell_smoke_scene(0.5, 4.5, 0.7, n=64, seed=7)
    NPH, RES = 5_000_000, 1024
else:
    scene = sc.cornell_scene(0.05, 0.5, 0.0)
    NPH, RES = 1_000_000, 512
out = {}
for it in its:
    R = bre.beam_radius_at(0.01, 0.5, it)
    with bre.BeamGather(0, timing=True) as g:
        for k, v in opts:
            g.set_option(k, v)
        g.trace_photons(scene, NPH, it, 5, R)
        g.camera_pass(scene, RES, RES, it, 5, True, True)
        ld = torch.zeros((RES * RES, 3), dtype=torch.float32, device="cuda")
        g.gather_camera(R, ld)
        g.synchronize()
        st = g.stats()
    L = max(st["beam_evals"], 1)
    rec = {"workload": wl, "iteration": it, "gather_ms": st["gather_ms"], "leaf_visits": st["beam_evals"],
           "on_lanes_per_leaf": st["candidates"] / L, "kept_beams_per_leaf": st["contributions"] / L,
           "scan_steps_per_leaf": st["node_visits"] / L, "min_on_kept_per_leaf": st["prefilter_rejects"] / L,
           "pair_compaction_steps_per_leaf": st["leaf_visits"] / L, "queued_pairs_per_leaf": st["useful_beam_evals"] / L,
           "transposed_frac": st["ccp_wave_evals"] / L}
    out[it] = rec
    print(json.dumps(rec), flush=True)
