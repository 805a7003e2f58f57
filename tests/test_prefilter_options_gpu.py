"""The tile kernel's prefilter variants give the SAME per-segment results, bit for bit.

Option 111 (prefilter margins: 1 = the round-3 rounding analysis, default; 0 = round 2's wider
margins) and option 112 (the per-lane tile line reject: 1 = on, default since round 4; 0 = off) only
change which NON-contributing (lane, beam) pairs reach the exact stage: a pair either margin rejects
has every reference-computed distance >= R + r (tests/test_margin_bound.py), and a lane the tile line
reject takes off a tile has no pair in it that can contribute (bre_gather.hip, above k_tile_axis).  Removing non-contributing pairs
from the beam-major queue leaves the contributing pairs in the same relative order, so every
per-segment sum and contribution count must be identical in all combinations -- on real C2
data (the production configuration: kernel 0, counters off, segment sort on) at a large and a small
radius."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W = H = 256
PHOTONS = 300_000


@pytest.mark.parametrize("medium,iteration", [("fog", 0), ("fog", 12), ("smoke", 0), ("smoke", 9)])
def test_prefilter_options_are_bit_identical(bre, scene_mod_gpu, medium, iteration):
    import torch

    scene = (scene_mod_gpu.cornell_scene(0.05, 0.5, 0.0) if medium == "fog" else
             scene_mod_gpu.cornell_smoke_scene(0.5, 4.5, 0.7, n=64, seed=7))
    R = bre.beam_radius_at(0.01, 0.5, iteration)
    out = {}
    for margin in (1, 0):
        for axis in (0, 1):
            with bre.BeamGather(0) as g:
                g.set_option(111, margin)
                g.set_option(112, axis)
                g.trace_photons(scene, PHOTONS, iteration, 5, R)
                n = g.camera_pass(scene, W, H, iteration, 5, True, True)
                rgb = torch.zeros((n, 3), dtype=torch.float32, device="cuda")
                cnt = torch.zeros((n, 2), dtype=torch.int32, device="cuda")
                g.gather_camera_segments(R, seg_rgb=rgb, counts=cnt)
                g.synchronize()
                out[(margin, axis)] = (rgb.cpu().numpy(), cnt.cpu().numpy())
    ref_rgb, ref_cnt = out[(1, 0)]
    assert ref_cnt[:, 1].sum() > 200_000  # a dense gather
    for key, (rgb, cnt) in out.items():
        assert np.array_equal(cnt, ref_cnt), key
        assert np.array_equal(rgb.view(np.uint32), ref_rgb.view(np.uint32)), key
