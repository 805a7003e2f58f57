"""The drop-in boundary (include/bre.h) on the GPU, round 3:

* bre_gather / bre_gather_device hand the caller's segments to the production kernel in the
  coherence order bre_gather_camera uses (BRE_OPT_SORT_SEGMENTS) and scatter the per-segment outputs
  back: exact contribution counts against the oracle, the same film with the sort on and off;
* a gather whose partial sums exceed the per-launch cap runs as several launches over whole-packet
  ranges, with per-segment sums bit-identical to one launch;
* packet shards with per-segment outputs define every entry (the other shards' entries are 0) and
  sum to the one-shard outputs;
* bre_gather_sharded (N contexts, here all on GPU 0): the same per-segment sums bit for bit as one
  context (each segment is gathered in the same packet), the film within float order;
* kernel 5 counts contributions without BRE_OPT_COUNTERS.
Reference: the gather loop photonbeam.cpp:494-508, batched (the result never feeds back, :510)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rel_l2(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def _seg_err(gpu, ref):
    scale = np.maximum(np.abs(ref).max(axis=1), 1e-30)
    return float((np.abs(gpu - ref).max(axis=1) / scale).max())


def _mixed(synth, nb=3000, w=48, h=40, nbounce=2500, seed=11):
    beams = synth.fog_beams(nb, seed=seed)
    cam = synth.camera_segments(w, h, seed=seed + 1)
    bnc = synth.bounce_segments(nbounce, seed=seed + 2, npix=w * h)
    segs = {k: np.concatenate([cam[k], bnc[k]]) for k in cam}
    # recorder order of the reference's camera walk: a pixel's depths next to each other
    order = np.argsort(segs["pixel"], kind="stable")
    return beams, {k: np.ascontiguousarray(v[order]) for k, v in segs.items()}, w * h


@pytest.mark.parametrize("sort", [1, 0])
def test_gather_sorts_and_scatters_back(bre, synth, oracle, sort):
    beams, segs, npix = _mixed(synth)
    R = 0.012
    ref = oracle.build(beams).gather(segs, R, npix=npix)
    accum = np.zeros((npix, 3), np.float32)
    with bre.BeamGather(0) as g:
        g.set_option(bre.OPT_SORT_SEGMENTS, sort)
        g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
        out = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], segs["pixel"], R=R, npix=npix, accum=accum,
                       counts=True)
    assert (out["counts"][:, 0] == -1).all()
    assert np.array_equal(out["counts"][:, 1], ref["contrib"])
    assert _seg_err(out["seg_rgb"], ref["seg_rgb"]) <= 1e-5
    assert _rel_l2(accum, ref["accum"]) <= 1e-6


def test_gather_device_sorted_equals_host_gather(bre, synth, oracle):
    import torch

    beams, segs, npix = _mixed(synth, seed=21)
    R = 0.01
    ref = oracle.build(beams).gather(segs, R, npix=npix)
    d = {k: torch.from_numpy(v).cuda().contiguous() for k, v in segs.items()}
    n = segs["tmax"].shape[0]
    acc = torch.zeros((npix, 3), dtype=torch.float32, device="cuda")
    rgb = torch.full((n, 3), float("nan"), dtype=torch.float32, device="cuda")
    cnt = torch.full((n, 2), -7, dtype=torch.int32, device="cuda")
    with bre.BeamGather(0) as g:
        g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
        g.gather_device(d["o"], d["p"], d["d"], d["tmax"], d["pixel"], R, npix, accum=acc, seg_rgb=rgb, counts=cnt)
        g.synchronize()
        host = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=R, counts=True)
    rgb, cnt = rgb.cpu().numpy(), cnt.cpu().numpy()
    assert np.array_equal(cnt[:, 1], ref["contrib"])
    assert np.array_equal(rgb, host["seg_rgb"])  # same sorted packets: bit-identical sums
    assert _rel_l2(acc.cpu().numpy(), ref["accum"]) <= 1e-6


@pytest.mark.parametrize("counts", [False, True])
def test_partial_cap_splits_launches_bit_identically(bre, synth, counts):
    beams, segs, npix = _mixed(synth, nb=4000, seed=31)
    R = 0.015
    res = []
    for cap_mib in (0, 1):  # 0: the default cap (one launch); 1 MiB: 320 (or 192) segments per launch
        with bre.BeamGather(0) as g:
            if cap_mib:
                g.set_option(109, cap_mib)
            g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
            res.append(g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=R, counts=counts))
    assert segs["tmax"].shape[0] > 10 * 320
    assert np.array_equal(res[0]["seg_rgb"], res[1]["seg_rgb"])
    if counts:
        assert np.array_equal(res[0]["counts"], res[1]["counts"])


def test_packet_shard_outputs_are_defined_and_sum(bre, synth):
    import torch

    beams, segs, npix = _mixed(synth, seed=41)
    R = 0.012
    n = segs["tmax"].shape[0]
    d = {k: torch.from_numpy(v).cuda().contiguous() for k, v in segs.items()}
    world = 3
    outs = []
    for rank in range(-1, world):
        rgb = torch.full((n, 3), float("nan"), dtype=torch.float32, device="cuda")
        cnt = torch.full((n, 2), -7, dtype=torch.int32, device="cuda")
        with bre.BeamGather(0) as g:
            if rank >= 0:
                g.set_shard(rank, world, 1, packets=True)
            g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
            g.gather_device(d["o"], d["p"], d["d"], d["tmax"], None, R, 0, seg_rgb=rgb, counts=cnt)
            g.synchronize()
        outs.append((rgb.cpu().numpy(), cnt.cpu().numpy()))
    one_rgb, one_cnt = outs[0]
    assert not np.isnan(one_rgb).any()
    owned = np.zeros(n, np.int32)
    for rgb, cnt in outs[1:]:
        assert not np.isnan(rgb).any() and not (cnt == -7).any()  # every entry written
        mine = cnt[:, 0] == -1  # the shard's own entries carry C = -1; the rest were zeroed
        owned += mine
        assert not rgb[~mine].any() and not cnt[~mine].any()
        assert np.array_equal(rgb[mine], one_rgb[mine]) and np.array_equal(cnt[mine], one_cnt[mine])
    assert (owned == 1).all()


def test_empty_beams_zero_through_the_index(bre, synth):
    import torch

    segs = synth.camera_segments(16, 8, seed=3)
    n = segs["tmax"].shape[0]
    d = {k: torch.from_numpy(v).cuda().contiguous() for k, v in segs.items()}
    rgb = torch.full((n, 3), float("nan"), dtype=torch.float32, device="cuda")
    with bre.BeamGather(0) as g:
        g.set_shard(1, 2, 1, packets=True)
        g.set_beams(np.zeros((0, 3)), np.zeros((0, 3)), np.zeros(0), np.zeros((0, 3)))
        g.gather_device(d["o"], d["p"], d["d"], d["tmax"], None, 0.01, 0, seg_rgb=rgb)
        g.synchronize()
    assert not rgb.isnan().any() and not rgb.any()


@pytest.mark.parametrize("nctx", [2, 3, 8])
def test_gather_sharded_equals_one_context(bre, synth, oracle, nctx):
    beams, segs, npix = _mixed(synth, nb=5000, w=64, h=48, nbounce=6000, seed=51)
    R = 0.011
    ref = oracle.build(beams).gather(segs, R, npix=npix)
    one_acc = np.zeros((npix, 3), np.float32)
    with bre.BeamGather(0) as g:
        g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
        one = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], segs["pixel"], R=R, npix=npix, accum=one_acc,
                       counts=True)
    ctxs = [bre.BeamGather(0) for _ in range(nctx)]
    try:
        bre.set_beams_sharded(ctxs, beams["start"], beams["end"], beams["radius"], beams["power"])
        acc = one_acc.copy()  # += semantics: the result is twice the one-context film
        out = bre.gather_sharded(ctxs, segs["o"], segs["p"], segs["d"], segs["tmax"], segs["pixel"], R=R,
                                 npix=npix, accum=acc, counts=True)
    finally:
        for c in ctxs:
            c.close()
    assert np.array_equal(out["counts"], one["counts"])
    assert np.array_equal(out["counts"][:, 1], ref["contrib"])
    assert np.array_equal(out["seg_rgb"], one["seg_rgb"])
    assert _rel_l2(acc, 2 * one_acc) <= 1e-6
    assert _rel_l2(acc, 2 * ref["accum"]) <= 1e-6


def test_gather_sharded_rejects_repeated_context(bre, synth):
    beams, segs, npix = _mixed(synth, nb=100, seed=61)
    g = bre.BeamGather(0)
    try:
        with pytest.raises(bre.BreError, match="repeated"):
            bre.set_beams_sharded([g, g], beams["start"], beams["end"], beams["radius"], beams["power"])
    finally:
        g.close()


def test_kernel5_counts_without_counters(bre, synth, oracle):
    beams, segs, npix = _mixed(synth, nb=2000, seed=71)
    R = 0.012
    ref = oracle.build(beams).gather(segs, R)
    with bre.BeamGather(0, kernel=5, counters=False) as g:
        g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
        out = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=R, counts=True)
    assert (out["counts"][:, 0] == -1).all()
    assert np.array_equal(out["counts"][:, 1], ref["contrib"])
    assert _seg_err(out["seg_rgb"], ref["seg_rgb"]) <= 1e-5
