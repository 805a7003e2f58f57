"""Stakes of the WorldBound sqrt reading (photonbeambvh.h:67-69):
C2 iterations 0 and 15 gathered with BRE_OPT_SQRT_MODE 0 (`sqrt` -> ::sqrt(double), the libstdc++
reading this build uses) and 1 (sqrtf), counters on: total candidates (beams whose box passes the
reference test), contributions, and the film difference.
    python profiles/r3/sqrt_mode.py [iterations, e.g. 0,15]"""
import importlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
bre = importlib.import_module("beam-radiance-estimate-pbrt_amd")
sc = importlib.import_module("beam-radiance-estimate-pbrt_amd.scene")
its = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,15").split(",")]
scene = sc.cornell_scene(0.05, 0.5, 0.0)
W = H = 512
out = {}
for it in its:
    R = bre.beam_radius_at(0.01, 0.5, it)
    res = {}
    for mode in (0, 1):
        with bre.BeamGather(0, counters=True, sqrt_mode=mode) as g:
            nb = g.trace_photons(scene, 1_000_000, it, 5, R)
            n = g.camera_pass(scene, W, H, it, 5, False, True)
            ld = torch.zeros((W * H, 3), dtype=torch.float32, device="cuda")
            cnt = torch.zeros((n, 2), dtype=torch.int32, device="cuda")
            g.gather_camera_segments(R, accum=ld, counts=cnt)
            g.synchronize()
            st = g.stats()
        res[mode] = {"beams": nb, "segments": n, "candidates": st["candidates"], "contributions": st["contributions"],
                     "film": ld.cpu().numpy().astype(np.float64), "counts": cnt.cpu().numpy()}
    a, b = res[0], res[1]
    dc = a["counts"] - b["counts"]
    rec = {"iteration": it, "beams": a["beams"], "segments": a["segments"],
           "candidates_mode0": a["candidates"], "candidates_mode1": b["candidates"],
           "candidate_diff": a["candidates"] - b["candidates"],
           "segments_with_candidate_diff": int((dc[:, 0] != 0).sum()),
           "contributions_mode0": a["contributions"], "contributions_mode1": b["contributions"],
           "segments_with_contribution_diff": int((dc[:, 1] != 0).sum()),
           "film_rel_l2": float(np.linalg.norm(a["film"] - b["film"]) / max(np.linalg.norm(a["film"]), 1e-300))}
    out[it] = rec
    print(json.dumps(rec), flush=True)
