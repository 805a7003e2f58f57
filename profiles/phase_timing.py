"""Per-phase cycle breakdown of the production tile kernel on real C2 iterations, from a
BRE_PHASE_TIMING=1 build (profiles/variant.sh phase "-DBRE_PHASE_TIMING=1"):
    BRE_LIBRARY=.../libbre_phase.so python profiles/phase_timing.py [c2|c3] [iterations...]
Sums over waves of s_memtime cycles: leaf staging (tile load, scan records, bundle test, LDS
stores), prefilter scan (queue pushes included, exact stage excluded), exact stage, whole wave."""
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
    tot = max(st["leaf_visits"], 1)
    rec = {"workload": wl, "iteration": it, "gather_ms": st["gather_ms"], "wave_cycles": st["leaf_visits"],
           "stage": st["candidates"] / tot, "scan": st["contributions"] / tot, "exact": st["node_visits"] / tot}
    rec["traversal_rest"] = 1 - rec["stage"] - rec["scan"] - rec["exact"]
    out[it] = rec
    print(json.dumps(rec), flush=True)
