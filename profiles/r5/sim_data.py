"""Real C2 inputs for the CPU funnel models (profiles/r3b/sim_funnel.py, profiles/r5/sim_bundle.py):
the oracle's photon pass (1M photons) and camera pass (512^2) at iteration IT, saved as
/tmp/c2_itIT.npz (bs, be, br: beams; so, sp, sd, st, sdep: camera segments; R).
usage: python profiles/r5/sim_data.py IT"""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle_lib import load_oracle  # noqa: E402

it = int(sys.argv[1])
bre = importlib.import_module("beam-radiance-estimate-pbrt_amd")
sc = importlib.import_module("beam-radiance-estimate-pbrt_amd.scene")
ora = load_oracle()
scene = sc.cornell_scene(0.05, 0.5, 0.0)
R = np.float32(bre.beam_radius_at(0.01, 0.5, it))
b = ora.trace_photons(scene, 1_000_000, iteration=it, max_depth=5, radius=R)
c = ora.camera_pass(scene, 512, 512, iteration=it, max_depth=5)
print({k: getattr(v, "shape", v) for k, v in c.items()})
dep = c.get("depth", np.zeros(c["tmax"].shape[0], np.int32))
np.savez(f"/tmp/c2_it{it}.npz", bs=b["start"], be=b["end"], br=b["radius"], so=c["o"], sp=c["p"], sd=c["d"],
         st=c["tmax"], sdep=dep, R=R)
print("beams", b["radius"].shape[0], "segments", c["tmax"].shape[0], "R", float(R))
