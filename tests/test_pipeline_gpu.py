"""Two libbre contexts on two HIP streams with iterations alternating between them (bench.py
--pipeline 1): iteration k+1's photon pass, BVH build and camera pass overlap iteration k's gather.
The iterations are independent (the gather never feeds back, photonbeam.cpp:510), so the summed films
equal a one-context sequential render to float summation order."""
import importlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_two_stream_pipeline_equals_sequential(bre):
    import torch

    sc = importlib.import_module("beam-radiance-estimate-pbrt_amd.scene")
    scene = sc.cornell_scene(0.05, 0.5, 0.0)
    W, H, photons, iters = 192, 160, 150_000, 4

    def run(nctx):
        ctxs = []
        for _ in range(nctx):
            g = bre.BeamGather(0)
            st = torch.cuda.Stream()
            g.set_stream(st.cuda_stream)
            ctxs.append((g, st))
        films = [torch.zeros((W * H, 3), dtype=torch.float32, device="cuda") for _ in range(nctx)]
        for it in range(iters):
            g, st = ctxs[it % nctx]
            R = bre.beam_radius_at(0.01, 0.5, it)
            with torch.cuda.stream(st):
                g.trace_photons(scene, photons, it, 5, R)
                g.camera_pass(scene, W, H, it, 5, True, True, surface=films[it % nctx])
                g.gather_camera(R, films[it % nctx])
        torch.cuda.synchronize()
        out = sum(f.double() for f in films).cpu().numpy()
        for g, _ in ctxs:
            g.synchronize()
            g.close()
        return out

    want, got = run(1), run(2)
    assert np.abs(want).max() > 0
    rel = np.sqrt(((got - want) ** 2).sum() / (want ** 2).sum())
    assert rel <= 1e-6, rel
