"""Stream order of the passes towards the caller's stream (include/bre.h, bre_set_stream).

The photon pass (with its BVH build) and the camera pass run on an internal stream of the device's
highest priority (internal option 117, on by default), forked from the caller's stream and joined back.
What the caller queued before a pass must be seen by it (a film written on the caller's stream right
before bre_camera_pass), and what the caller queues after it must see the pass's results (a clone of
the film right after the call; the film freed and its memory reused by the torch caching allocator
right after the call).  The results must be the same bits with the option on and off."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W = H = 64


def _run(bre, scene, prio, reuse):
    import torch

    it, R = 1, bre.beam_radius_at(0.01, 0.5, 1)
    with bre.BeamGather(0) as g:
        g.set_option(117, prio)
        st = torch.cuda.Stream()
        g.set_stream(st.cuda_stream)
        with torch.cuda.stream(st):
            seed = torch.full((W * H, 3), 0.25, dtype=torch.float32, device="cuda")
            g.trace_photons(scene, 20_000, it, 5, R)
            # queued on the caller's stream right before the pass: the pass must add onto 0.25
            surf = seed.clone()
            n = g.camera_pass(scene, W, H, it, 5, True, True, surface=surf)
            surf_copy = surf.clone()  # queued after the pass: sees its writes
            film = torch.zeros((W * H, 3), dtype=torch.float32, device="cuda")
            if reuse:
                del surf  # its block goes back to the caching allocator at once ...
                junk = torch.full((W * H, 3), -7.0, dtype=torch.float32, device="cuda")  # ... and is reused
                junk.add_(1.0)
            g.gather_camera(R, film)
            out = (surf_copy.clone(), film.clone())
        st.synchronize()
        g.synchronize()
        return n, out[0].cpu().numpy(), out[1].cpu().numpy()


@pytest.mark.parametrize("prio", [1, 0])
def test_passes_keep_caller_stream_order(bre, scene_mod_gpu, prio):
    scene = scene_mod_gpu.cornell_scene(0.05, 0.5, 0.0)
    n0, s0, f0 = _run(bre, scene, prio, reuse=False)
    n1, s1, f1 = _run(bre, scene, prio, reuse=True)
    assert n0 == n1 and n0 > 0
    assert np.array_equal(s0, s1) and np.array_equal(f0, f1)
    # the pass added onto the value the caller wrote before it: every pixel >= 0.25, some above
    assert (s0 >= 0.25).all() and (s0 > 0.25).any()
    assert np.abs(f0).sum() > 0


def test_pass_stream_option_gives_the_same_bits(bre, scene_mod_gpu):
    scene = scene_mod_gpu.cornell_scene(0.05, 0.5, 0.0)
    a = _run(bre, scene, 1, reuse=True)
    b = _run(bre, scene, 0, reuse=True)
    assert a[0] == b[0] and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
