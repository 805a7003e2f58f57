"""SHA-1 of per-segment seg_rgb (deterministic per segment; the film's per-pixel global atomics are
not) for fixed synthetic beams and segments, from the libbre named by BRE_LIBRARY."""
import hashlib
import importlib
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
bre = importlib.import_module("beam-radiance-estimate-pbrt_amd")
synth = importlib.import_module("beam-radiance-estimate-pbrt_amd.synth")
out = []
for kind in ("camera", "bounce", "long"):
    if kind == "long":
        beams = synth.fog_beams(6000, seed=81, radius=0.05, mean_length=0.8)
        segs = synth.bounce_segments(6000, seed=82)
        R = 0.08
    else:
        beams = synth.fog_beams(200000, seed=83)
        segs = synth.camera_segments(128, 128, seed=84) if kind == "camera" else synth.bounce_segments(16384, seed=85)
        R = 0.01
    with bre.BeamGather(0, counters=False, kernel=0) as g:
        g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
        o = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=R, counts=True)
    out.append(f"{kind}:{hashlib.sha1(np.ascontiguousarray(o['seg_rgb']).tobytes()).hexdigest()[:12]}:{int(o['counts'][:, 1].sum())}")
print(" ".join(out))
