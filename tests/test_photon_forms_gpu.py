"""The photon pass's single-trace form (per-photon beam slots, then a copy to the photon-major
offsets, and a re-trace of only the photons with more beams than slots) gives the SAME beam array,
bit for bit and in the same order, as the two-trace form (count, scan, re-trace every photon) --
bre_photon.hip, option 116.  Forced slot counts of 2 and 3 make many photons overflow, so the
overflow re-trace is exercised; the default (64 slots at these photon counts) rarely overflows.
Both are checked against the recursive CPU restatement in tests/test_photon_gpu.py."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("medium", ["fog", "smoke"])
def test_photon_forms_bit_identical(bre, scene_mod_gpu, medium):
    scene = (scene_mod_gpu.cornell_scene(0.05, 0.5, 0.0) if medium == "fog" else
             scene_mod_gpu.cornell_smoke_scene(0.5, 4.5, 0.7, n=32, seed=3))
    out = {}
    for mode in (0, 1, 2, 3):  # two traces, single trace (auto slots), 2 and 3 forced slots
        with bre.BeamGather(0) as g:
            g.set_option(116, mode)
            n = g.trace_photons(scene, 200_000, 4, 5, 0.01)
            out[mode] = (n, g.get_beams())
    n0, ref = out[0]
    assert n0 > 400_000  # > 2 beams per photon on average: forced 2 / 3 slots overflow often
    for mode, (n, b) in out.items():
        assert n == n0, mode
        for k in ("start", "end", "radius", "power"):
            assert np.array_equal(b[k].view(np.uint32), ref[k].view(np.uint32)), (mode, k)
