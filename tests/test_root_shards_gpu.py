"""Work-root shards (BRE_OPT_SHARD_MODE 2, bench.py --shard-mode roots): every shard runs the whole
camera pass and gathers EVERY segment against its own work roots (rank, rank + count, ... of the
size-ordered list), so a rank's waves sweep whole subtrees with all packets, as one GPU does.  The
shards' contribution counts must add up to the one-shard counts exactly (each (segment, beam) pair
lies in exactly one subtree), and their per-segment sums and films to the one-shard ones within
float32 summation tolerance (the subtree partials are added in another grouping)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("count", [3, 8])
def test_root_shards_sum_to_one_shard(bre, scene_mod_gpu, count):
    import torch

    scene = scene_mod_gpu.cornell_scene(0.05, 0.5, 0.0)
    it = 2
    R = bre.beam_radius_at(0.01, 0.5, it)
    W = H = 192

    def run(rank, cnt):
        with bre.BeamGather(0) as g:
            if cnt > 1:
                g.set_shard(rank, cnt, roots=True)
            g.trace_photons(scene, 200_000, it, 5, R)
            n = g.camera_pass(scene, W, H, it, 5, True, True)
            rgb = torch.zeros((n, 3), dtype=torch.float32, device="cuda")
            cnts = torch.zeros((n, 2), dtype=torch.int32, device="cuda")
            film = torch.zeros((W * H, 3), dtype=torch.float32, device="cuda")
            g.gather_camera_segments(R, film, seg_rgb=rgb, counts=cnts)
            g.synchronize()
            return rgb.cpu().numpy().astype(np.float64), cnts.cpu().numpy(), film.cpu().numpy().astype(np.float64)

    rgb1, cnt1, film1 = run(0, 1)
    assert cnt1[:, 1].sum() > 50_000
    parts = [run(r, count) for r in range(count)]
    cnt = sum(p[1][:, 1].astype(np.int64) for p in parts)
    assert np.array_equal(cnt, cnt1[:, 1])
    rgb = sum(p[0] for p in parts)
    n = np.maximum(cnt1[:, 1], 1).astype(np.float64)[:, None]
    tol = np.maximum(1e-5, 4 * 2.0 ** -24 * np.sqrt(n))
    assert (np.abs(rgb - rgb1) <= tol * np.abs(rgb1) + 1e-30).all()
    film = sum(p[2] for p in parts)
    assert np.linalg.norm(film - film1) <= 1e-5 * np.linalg.norm(film1)
