"""Gather cost by camera-path depth and segment sort key (round 3): the camera segments of one C2 /
C3 iteration, split into depth 0 (primary rays), depth >= 1 (bounces) and all, each gathered through
bre_gather_device (which coherence-sorts them with sort key mode K, libbre option 105) with timing,
then once more with counters for the work counts.
    python profiles/r3/depth_keys.py [c2|c3] [iteration] [keys, e.g. 1,2,3]"""
import importlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
bre = importlib.import_module("beam-radiance-estimate-pbrt_amd")
sc = importlib.import_module("beam-radiance-estimate-pbrt_amd.scene")

wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
it = int(sys.argv[2]) if len(sys.argv) > 2 else 0
keys = [int(k) for k in (sys.argv[3] if len(sys.argv) > 3 else "1,2,3").split(",")]
if wl == "c3":
    scene, NPH, RES = sc.cornell_smoke_scene(0.5, 4.5, 0.7, n=64, seed=7), 5_000_000, 1024
else:
    scene, NPH, RES = sc.cornell_scene(0.05, 0.5, 0.0), 1_000_000, 512
R = bre.beam_radius_at(0.01, 0.5, it)
out = {"workload": wl, "iteration": it, "R": R}
with bre.BeamGather(0, timing=True) as g:
    g.trace_photons(scene, NPH, it, 5, R)
    g.camera_pass(scene, RES, RES, it, 5, True, True)
    s = g.get_segments()
    dev = torch.device("cuda")
    subsets = {"all": np.ones_like(s["depth"], bool), "depth0": s["depth"] == 0, "depth1+": s["depth"] >= 1}
    for key in keys:
        g.set_option(105, key)
        for name, m in subsets.items():
            idx = np.nonzero(m)[0]
            t = {k: torch.from_numpy(np.ascontiguousarray(s[k][idx])).to(dev) for k in ("o", "p", "d", "tmax", "pixel")}
            acc = torch.zeros((RES * RES, 3), dtype=torch.float32, device=dev)
            rec = {"key": key, "segments": int(len(idx))}
            for counters in (False, False, True):
                g.set_option(bre.OPT_COUNTERS, int(counters))
                g.gather_device(t["o"], t["p"], t["d"], t["tmax"], t["pixel"], R, RES * RES, accum=acc)
                g.synchronize()
                st = g.stats()
                n = max(len(idx), 1)
                if not counters:
                    rec["gather_ms"] = st["gather_ms"]
                    rec["estimates_per_s"] = n / (st["gather_ms"] * 1e-3)
                else:
                    rec["contributions_per_estimate"] = st["contributions"] / n
                    rec["staged_per_packet"] = st["beam_evals"] / (n / 64)
                    rec["kept_per_packet"] = st["useful_beam_evals"] / (n / 64)
                    rec["bundle_keep_frac"] = st["useful_beam_evals"] / max(st["beam_evals"], 1)
                    rec["queued_per_segment"] = st["queued_pairs"] / n
                    rec["tests_per_queued"] = st["useful_beam_evals"] * 64 / max(st["queued_pairs"], 1)
                    rec["node_visits_per_packet"] = st["node_visits"] / (n / 64)
            g.set_option(bre.OPT_COUNTERS, 0)
            out[f"{name}/k{key}"] = rec
            print(name, json.dumps(rec), flush=True)
print(json.dumps(out))
