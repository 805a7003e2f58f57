"""Per-segment sums of the default library against another build on the same inputs (bit for bit):
    python profiles/r3b/bitcmp.py dump OUT.npz [workload]   (BRE_LIBRARY selects the build)
    python profiles/r3b/bitcmp.py cmp A.npz B.npz
Runs the C2 (or C3) camera segments of iterations 0, 8 and 15 (C3: 0) through bre_gather_camera_segments."""
import importlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

if sys.argv[1] == "cmp":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    for k in a.files:
        same = np.array_equal(a[k].view(np.uint32) if a[k].dtype == np.float32 else a[k],
                              b[k].view(np.uint32) if b[k].dtype == np.float32 else b[k])
        print(k, a[k].shape, "bit-identical" if same else "DIFFERENT (max rel %.3g)" % (
            np.max(np.abs(a[k].astype(np.float64) - b[k]) / np.maximum(np.abs(a[k].astype(np.float64)), 1e-30))))
    sys.exit(0)

import torch  # noqa: E402

bre = importlib.import_module("beam-radiance-estimate-pbrt_amd")
sc = importlib.import_module("beam-radiance-estimate-pbrt_amd.scene")
wl = sys.argv[3] if len(sys.argv) > 3 else "c2"
if wl == "c3":
    scene, NPH, RES = sc.cornell_smoke_scene(0.5, 4.5, 0.7, n=64, seed=7), 5_000_000, 1024
else:
    scene, NPH, RES = sc.cornell_scene(0.05, 0.5, 0.0), 1_000_000, 512
out = {}
for it in ([0] if wl == "c3" else [0, 8, 15]):
    R = bre.beam_radius_at(0.01, 0.5, it)
    with bre.BeamGather(0) as g:
        g.trace_photons(scene, NPH, it, 5, R)
        n = g.camera_pass(scene, RES, RES, it, 5, True, True)
        rgb = torch.zeros((n, 3), dtype=torch.float32, device="cuda")
        cnt = torch.zeros((n, 2), dtype=torch.int32, device="cuda")
        g.gather_camera_segments(R, seg_rgb=rgb, counts=cnt)
        g.synchronize()
        out[f"rgb{it}"] = rgb.cpu().numpy()
        out[f"cnt{it}"] = cnt.cpu().numpy()
np.savez(sys.argv[2], **out)
print("dumped", {k: v.shape for k, v in out.items()})
