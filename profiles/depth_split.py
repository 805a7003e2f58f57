"""Gather cost by camera-path depth: the camera segments of one C2 / C3 iteration split into depth 0
(primary rays, coherent) and depth >= 1 (bounce rays), each subset coherence-sorted on the host with a
6-D Morton key of (origin, end point) like bre_sort.hip, then gathered through bre_gather_device with
timing (and once more with counters for the work counts).
    python profiles/depth_split.py [c2|c3] [iteration]"""
import importlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
bre = importlib.import_module("beam-radiance-estimate-pbrt_amd")
sc = importlib.import_module("beam-radiance-estimate-pbrt_amd.scene")

wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
it = int(sys.argv[2]) if len(sys.argv) > 2 else 0
if wl == "c3":
    scene, NPH, RES = sc.cornell_smoke_scene(0.5, 4.5, 0.7, n=64, seed=7), 5_000_000, 1024
else:
    scene, NPH, RES = sc.cornell_scene(0.05, 0.5, 0.0), 1_000_000, 512
R = bre.beam_radius_at(0.01, 0.5, it)


def morton6(o, p):
    pts = np.concatenate([o, p], axis=1).astype(np.float64)
    lo, hi = pts.min(axis=0), pts.max(axis=0)
    q = ((pts - lo) / np.maximum(hi - lo, 1e-30) * 1023).astype(np.uint64)
    key = np.zeros(len(pts), np.uint64)
    for b in range(10):
        for a in range(6):
            key |= ((q[:, a] >> np.uint64(b)) & np.uint64(1)) << np.uint64(6 * b + a)
    return np.argsort(key, kind="stable")


out = {"workload": wl, "iteration": it, "R": R}
with bre.BeamGather(0, timing=True) as g:
    g.trace_photons(scene, NPH, it, 5, R)
    g.camera_pass(scene, RES, RES, it, 5, True, True)
    s = g.get_segments()
    dev = torch.device("cuda")
    subsets = {"all": np.ones_like(s["depth"], bool), "depth0": s["depth"] == 0, "depth1+": s["depth"] >= 1}
    for name, m in subsets.items():
        idx = np.nonzero(m)[0]
        idx = idx[morton6(s["o"][idx], s["p"][idx])]
        t = {k: torch.from_numpy(np.ascontiguousarray(s[k][idx])).to(dev) for k in ("o", "p", "d", "tmax", "pixel")}
        acc = torch.zeros((RES * RES, 3), dtype=torch.float32, device=dev)
        rec = {"segments": int(len(idx))}
        for counters in (False, True):
            g.set_option(bre.OPT_COUNTERS, int(counters))
            g.gather_device(t["o"], t["p"], t["d"], t["tmax"], t["pixel"], R, RES * RES, accum=acc)
            g.synchronize()
            st = g.stats()
            if not counters:
                rec["gather_ms"] = st["gather_ms"]
                rec["estimates_per_s"] = len(idx) / (st["gather_ms"] * 1e-3)
            else:
                n = max(len(idx), 1)
                rec["candidates_per_estimate"] = st["candidates"] / n
                rec["contributions_per_estimate"] = st["contributions"] / n
                rec["staged_per_packet"] = st["beam_evals"] / (n / 64)
                rec["kept_per_packet"] = st["useful_beam_evals"] / (n / 64)
                rec["bundle_keep_frac"] = st["useful_beam_evals"] / max(st["beam_evals"], 1)
                rec["exact_pairs_per_segment"] = st["ccp_wave_evals"] * 64 / n
        g.set_option(bre.OPT_COUNTERS, 0)
        out[name] = rec
        print(name, json.dumps(rec), flush=True)
print(json.dumps(out))
