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


@pytest.mark.parametrize("kernel", [2, 5])
def test_root_shards_refuse_kernels_without_work_roots(bre, scene_mod_gpu, kernel):
    """Kernels 2 and 5 have no work roots to split: under work-root shards every shard would gather
    every pair (films summing to count x the image), so the gather is refused with BRE_ERR_STATE."""
    import torch

    scene = scene_mod_gpu.cornell_scene(0.05, 0.5, 0.0)
    with bre.BeamGather(0, kernel=kernel) as g:
        g.set_shard(1, 3, roots=True)
        g.trace_photons(scene, 5000, 0, 5, 0.02)
        n = g.camera_pass(scene, 32, 32, 0, 5, True, True)
        assert n > 0
        film = torch.zeros((32 * 32, 3), dtype=torch.float32, device="cuda")
        with pytest.raises(bre.BreError) as e:
            g.gather_camera(0.02, film)
            g.synchronize()
        assert e.value.status == 4


def test_root_shards_with_the_xcd_block_map(bre, scene_mod_gpu):
    """3 work-root shards split S = 256 roots into 86 per shard, not a multiple of 8: block map 0 (the
    XCD map, option 107) would leave roots unassigned, so such a launch takes the LPT map -- the shards'
    contribution counts still add up to the one-shard counts."""
    import torch

    scene = scene_mod_gpu.cornell_scene(0.05, 0.5, 0.0)
    R = bre.beam_radius_at(0.01, 0.5, 1)

    def counts(rank, cnt):
        with bre.BeamGather(0) as g:
            g.set_option(107, 0)
            if cnt > 1:
                g.set_shard(rank, cnt, roots=True)
            g.trace_photons(scene, 100_000, 1, 5, R)
            n = g.camera_pass(scene, 96, 96, 1, 5, True, True)
            cnts = torch.zeros((n, 2), dtype=torch.int32, device="cuda")
            rgb = torch.zeros((n, 3), dtype=torch.float32, device="cuda")
            g.gather_camera_segments(R, None, seg_rgb=rgb, counts=cnts)
            g.synchronize()
            return cnts.cpu().numpy()[:, 1].astype(np.int64)

    one = counts(0, 1)
    assert one.sum() > 10_000
    assert np.array_equal(sum(counts(r, 3) for r in range(3)), one)


def test_empty_packet_shard_on_a_fresh_context(bre, scene_mod_gpu):
    """A packet shard that gets no packet (more shards than packets) never launches the gather: its film
    compose must still have the context's flags word (it used to read a null counter block)."""
    import torch

    scene = scene_mod_gpu.cornell_scene(0.05, 0.5, 0.0)
    with bre.BeamGather(0) as g:
        g.set_shard(7, 8, packets=True)
        g.trace_photons(scene, 5000, 0, 5, 0.02)
        n = g.camera_pass(scene, 8, 8, 0, 5, True, True)
        assert 0 < n <= 7 * 64 and bre.shard_segments(n, 7, 8, 1) == 0
        film = torch.zeros((64, 3), dtype=torch.float32, device="cuda")
        g.gather_camera(0.02, film)
        g.synchronize()
        assert float(film.abs().sum()) == 0.0  # no segment of this shard (the surfaces went nowhere: no buffer)


def test_root_shards_refuse_film_classes(bre, scene_mod_gpu):
    """Packet-class films gather each rank's planes whole (dist.ShardedFrame._gather_planes): under
    work-root shards every rank writes partial sums into every plane, so the gather would drop most
    contributions.  The library refuses the combination with BRE_ERR_STATE, and so does
    ShardedFrame (tests/test_dist.py)."""
    import torch

    scene = scene_mod_gpu.cornell_scene(0.05, 0.5, 0.0)
    with bre.BeamGather(0) as g:
        g.set_shard(0, 2, roots=True)
        g.set_film_classes(bre.FILM_CLASSES)
        g.trace_photons(scene, 5000, 0, 5, 0.02)
        n = g.camera_pass(scene, 32, 32, 0, 5, True, True,
                          surface=torch.zeros((bre.FILM_CLASSES * 32 * 32, 3), dtype=torch.float32, device="cuda"))
        assert n > 0
        film = torch.zeros((bre.FILM_CLASSES * 32 * 32, 3), dtype=torch.float32, device="cuda")
        with pytest.raises(bre.BreError) as e:
            g.gather_camera(0.02, film)
            g.synchronize()
        assert e.value.status == 4  # BRE_ERR_STATE
