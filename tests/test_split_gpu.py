"""The tile kernel's work-root count S (BRE_OPT_SPLIT, powers of two up to 1024) only partitions the
tree: every segment's contributing pairs and counts are the same for any S, and its sum differs only
by the order in which k_reduce adds the S subtree partials (bre_gather.hip k_roots: size-balanced
roots, largest first).  Real C2 data at a large and a small radius."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("iteration", [0, 12])
def test_split_changes_no_contribution(bre, scene_mod_gpu, iteration):
    import torch

    scene = scene_mod_gpu.cornell_scene(0.05, 0.5, 0.0)
    R = bre.beam_radius_at(0.01, 0.5, iteration)
    out = {}
    for S in (1, 64, 256, 1024):
        with bre.BeamGather(0, split=S) as g:
            g.trace_photons(scene, 300_000, iteration, 5, R)
            n = g.camera_pass(scene, 256, 256, iteration, 5, True, True)
            rgb = torch.zeros((n, 3), dtype=torch.float32, device="cuda")
            cnt = torch.zeros((n, 2), dtype=torch.int32, device="cuda")
            g.gather_camera_segments(R, seg_rgb=rgb, counts=cnt)
            g.synchronize()
            out[S] = (rgb.cpu().numpy().astype(np.float64), cnt.cpu().numpy())
    ref_rgb, ref_cnt = out[256]
    assert ref_cnt[:, 1].sum() > 100_000
    for S, (rgb, cnt) in out.items():
        assert np.array_equal(cnt, ref_cnt), S
        # float32 sums of the same terms in another grouping: the production tests' bound, max(1e-5, 4u sqrt(n))
        n = np.maximum(ref_cnt[:, 1], 1).astype(np.float64)[:, None]
        tol = np.maximum(1e-5, 4 * 2.0 ** -24 * np.sqrt(n))
        assert (np.abs(rgb - ref_rgb) <= tol * np.abs(ref_rgb) + 1e-30).all(), S
