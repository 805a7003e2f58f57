"""GPU parity: libbre (HIP, gfx950) against the CPU oracle on the same seeded inputs.

Bar (DESIGN.md "parity contract"):
* candidate count C and contribution count per segment: EXACT (integer work: the candidate set is
  the reference's, pair by pair);
* per-segment RGB: relative error <= 1e-5 of the segment's magnitude (float summation order
  differs from the reference's DFS order; every individual pair is bit-identical);
* image: relative L2 <= 1e-3 (north star), in practice ~1e-7.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEG_RTOL = 1e-5


def _seg_close(gpu, ref, rtol=SEG_RTOL):
    scale = np.maximum(np.abs(ref).max(axis=1, keepdims=True), 1e-30)
    err = (np.abs(gpu - ref) / scale).max()
    return err


def _rel_l2(a, b):
    den = np.sqrt((b.astype(np.float64) ** 2).sum())
    return float(np.sqrt(((a.astype(np.float64) - b) ** 2).sum()) / max(den, 1e-300))


@pytest.fixture(scope="module")
def ctxs(bre):
    out = {}
    for k in (1, 2):
        out[k] = bre.BeamGather(0, counters=True, kernel=k)
    yield out
    for c in out.values():
        c.close()


@pytest.mark.parametrize("kernel", [0, 1, 2, 3, 4, 6])
@pytest.mark.parametrize("leaf", [1, 4, 8, 64])
def test_camera_segments_match_oracle(bre, synth, oracle, kernel, leaf):
    if kernel == 3 and leaf > 4:
        pytest.skip("kernel 3 needs leaf clusters <= 4 (tested in test_kernel3_rejects_large_leaves)")
    beams = synth.fog_beams(3000, seed=12345)
    segs = synth.camera_segments(48, 40, seed=777)
    R = 0.01
    ref = oracle.build(beams).gather(segs, R)
    with bre.BeamGather(0, counters=True, kernel=kernel, leaf_size=leaf) as g:
        g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
        out = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], segs["pixel"], R=R, counts=True)
        st = g.stats()
    assert np.array_equal(out["counts"][:, 0], ref["cand"]), "candidate sets differ"
    assert np.array_equal(out["counts"][:, 1], ref["contrib"]), "contribution sets differ"
    assert _seg_close(out["seg_rgb"], ref["seg_rgb"]) <= SEG_RTOL
    assert st["candidates"] == int(ref["cand"].sum())
    assert st["contributions"] == int(ref["contrib"].sum())


@pytest.mark.parametrize("kernel", [0, 1, 2, 3, 4, 6])
def test_bounce_segments_match_oracle(bre, synth, oracle, kernel):
    beams = synth.fog_beams(3000, seed=99)
    segs = synth.bounce_segments(3000, seed=5)
    R = 0.013
    ref = oracle.build(beams).gather(segs, R)
    with bre.BeamGather(0, counters=True, kernel=kernel, leaf_size=32 if kernel == 4 else None) as g:
        g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
        out = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], segs["pixel"], R=R, counts=True)
    assert np.array_equal(out["counts"][:, 0], ref["cand"])
    assert np.array_equal(out["counts"][:, 1], ref["contrib"])
    assert _seg_close(out["seg_rgb"], ref["seg_rgb"]) <= SEG_RTOL


def test_pixel_accumulation_and_image_l2(bre, synth, oracle):
    """Several segments per pixel (camera path depths) accumulate like PhotonBeamPixel::Ld."""
    beams = synth.fog_beams(2000, seed=3)
    cam = synth.camera_segments(32, 32, seed=4)
    bnc = synth.bounce_segments(2048, seed=6, npix=1024)
    segs = {k: np.concatenate([cam[k], bnc[k]]) for k in cam}
    R = 0.01
    ref = oracle.build(beams).gather(segs, R, npix=1024)
    accum = np.zeros((1024, 3), np.float32)
    with bre.BeamGather(0) as g:
        g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
        g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], segs["pixel"], R=R, npix=1024, accum=accum,
                 seg_rgb=False)
    assert _rel_l2(accum, ref["accum"]) <= 1e-6


def test_empty_beam_set(bre, synth):
    segs = synth.camera_segments(8, 8)
    accum = np.ones((64, 3), np.float32)
    with bre.BeamGather(0, counters=True) as g:
        g.set_beams(np.zeros((0, 3)), np.zeros((0, 3)), np.zeros(0), np.zeros((0, 3)))
        out = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], segs["pixel"], R=0.01, npix=64, accum=accum,
                       counts=True)
    assert not out["seg_rgb"].any() and not out["counts"].any()
    assert (accum == 1).all()


def test_single_beam_and_tiny_sets(bre, synth, oracle):
    for n in (1, 2, 3, 5, 17):
        beams = synth.fog_beams(n, seed=100 + n, mean_length=0.6)
        segs = synth.bounce_segments(2000, seed=n)
        ref = oracle.build(beams).gather(segs, 0.05)
        with bre.BeamGather(0, counters=True) as g:
            g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
            out = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=0.05, counts=True)
        assert np.array_equal(out["counts"][:, 0], ref["cand"]), n
        assert _seg_close(out["seg_rgb"], ref["seg_rgb"]) <= SEG_RTOL


def test_duplicate_centroids_use_group_box(bre, synth, oracle):
    """Beams with bit-identical centroids share one SAH leaf in the reference, whose union box is
    tested (photonbeambvh.cpp:289-297); libbre reproduces that with group boxes."""
    base = synth.fog_beams(400, seed=8, mean_length=0.3)
    start, end = base["start"].copy(), base["end"].copy()
    # mirror every 4th beam around its centre: same centroid, different (quirky) box
    idx = np.arange(0, 400, 4)
    rev_s, rev_e = end[idx].copy(), start[idx].copy()
    beams = {
        "start": np.concatenate([start, rev_s]), "end": np.concatenate([end, rev_e]),
        "radius": np.full(500, 0.02, np.float32),
        "power": np.concatenate([base["power"], base["power"][idx]]),
    }
    segs = synth.bounce_segments(3000, seed=9)
    bvh = oracle.build(beams)
    ref = bvh.gather(segs, 0.02)
    bf = oracle.bruteforce(beams, segs, 0.02)
    assert np.array_equal(ref["cand"], bf["cand"])
    with bre.BeamGather(0, counters=True) as g:
        g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
        out = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=0.02, counts=True)
    assert np.array_equal(out["counts"][:, 0], ref["cand"])
    assert np.array_equal(out["counts"][:, 1], ref["contrib"])


def test_axis_aligned_rays_and_degenerate_segments(bre, oracle):
    """Zero direction components (inf/NaN slab values) and zero-length segments."""
    rng = np.random.default_rng(1)
    n = 500
    start = rng.random((n, 3), dtype=np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d[::3, 0] = 0  # some axis-aligned beams
    end = (start + 0.2 * d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    beams = {"start": start, "end": end, "radius": np.full(n, 0.03, np.float32),
             "power": rng.random((n, 3), dtype=np.float32)}
    m = 3000
    o = np.round(rng.random((m, 3)) * 16).astype(np.float32) / 16  # origins on box planes often
    dd = rng.normal(size=(m, 3)).astype(np.float32)
    dd[0::2, 1] = 0.0
    dd[0::3, 2] = 0.0
    dd[5::7, 0] = -0.0
    dd /= np.maximum(np.linalg.norm(dd, axis=1, keepdims=True), 1e-6)
    t = rng.random(m).astype(np.float32)
    t[::11] = 0.0  # zero-length segments: p == o
    p = (o + dd * t[:, None]).astype(np.float32)
    segs = {"o": o, "p": p, "d": dd.astype(np.float32), "tmax": t}
    ref = oracle.build(beams).gather(segs, 0.02)
    with bre.BeamGather(0, counters=True) as g:
        g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
        for k in (0, 1, 2, 3, 4, 6):
            g.set_option(bre.OPT_KERNEL, k)  # the tree shape follows the kernel: rebuild
            g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
            out = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=0.02, counts=True)
            assert np.array_equal(out["counts"][:, 0], ref["cand"]), k
            assert np.array_equal(out["counts"][:, 1], ref["contrib"]), k
            assert _seg_close(out["seg_rgb"], ref["seg_rgb"]) <= SEG_RTOL


def test_zero_length_beams_never_gathered(bre, synth, oracle):
    beams = synth.fog_beams(300, seed=21)
    beams["end"][::10] = beams["start"][::10]  # WorldBound is NaN (0 * inf)
    segs = synth.bounce_segments(2000, seed=22)
    bf = oracle.bruteforce(beams, segs, 0.02)
    with bre.BeamGather(0, counters=True) as g:
        g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
        out = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=0.02, counts=True)
        assert g.stats()["n_beams_valid"] == 270
    assert np.array_equal(out["counts"][:, 0], bf["cand"])
    assert _seg_close(out["seg_rgb"], bf["seg_rgb"]) <= SEG_RTOL


def test_pixel_out_of_range_is_an_error(bre, synth):
    beams = synth.fog_beams(100)
    segs = synth.camera_segments(4, 4)
    with bre.BeamGather(0) as g:
        g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
        with pytest.raises(bre.BreError):
            g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], segs["pixel"], R=0.01, npix=8,
                     accum=np.zeros((8, 3), np.float32))


def test_device_api_matches_host_api(bre, synth):
    import torch

    beams = synth.fog_beams(5000, seed=31)
    segs = synth.camera_segments(64, 64, seed=32)
    dev = {k: torch.from_numpy(v).cuda().contiguous() for k, v in beams.items()}
    dseg = {k: torch.from_numpy(v).cuda().contiguous() for k, v in segs.items()}
    with bre.BeamGather(0) as g:
        g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
        host = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=0.01)["seg_rgb"]
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    with bre.BeamGather(0) as g:
        g.set_stream(stream.cuda_stream)
        g.set_beams_device(dev["start"], dev["end"], dev["radius"], dev["power"])
        out = torch.zeros((4096, 3), dtype=torch.float32, device="cuda")
        acc = torch.zeros((4096, 3), dtype=torch.float32, device="cuda")
        g.gather_device(dseg["o"], dseg["p"], dseg["d"], dseg["tmax"], dseg["pixel"], 0.01, 4096, accum=acc,
                        seg_rgb=out)
        torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), host)
    assert np.array_equal(acc.cpu().numpy(), host)  # one segment per pixel: single add each


def test_deterministic_per_segment(bre, synth):
    beams = synth.fog_beams(20000, seed=41)
    segs = synth.camera_segments(64, 64, seed=42)
    with bre.BeamGather(0) as g:
        g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
        a = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=0.01)["seg_rgb"]
        g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
        b = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=0.01)["seg_rgb"]
    assert np.array_equal(a, b)


@pytest.mark.parametrize("kernel", [0, 1, 3, 4, 6])
@pytest.mark.parametrize("split", [1, 2, 8, 64])
def test_subtree_split_matches_oracle(bre, synth, oracle, split, kernel):
    beams = synth.fog_beams(4000, seed=51)
    segs = synth.camera_segments(40, 36, seed=52)
    ref = oracle.build(beams).gather(segs, 0.01)
    with bre.BeamGather(0, counters=True, kernel=kernel, split=split) as g:
        g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
        out = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], segs["pixel"], R=0.01, counts=True)
    assert np.array_equal(out["counts"][:, 0], ref["cand"])
    assert np.array_equal(out["counts"][:, 1], ref["contrib"])
    assert _seg_close(out["seg_rgb"], ref["seg_rgb"]) <= SEG_RTOL


@pytest.mark.parametrize("kind", ["camera", "bounce", "long"])
def test_prefilter_changes_no_bit(bre, synth, kind):
    """The conservative line-distance reject must not drop any contributing pair: outputs with and
    without it are bit-identical, on coherent, incoherent and long-beam / large-radius inputs."""
    if kind == "long":
        beams = synth.fog_beams(6000, seed=61, radius=0.05, mean_length=0.8)
        segs = synth.bounce_segments(6000, seed=62)
        R = 0.08
    else:
        beams = synth.fog_beams(20000, seed=63)
        segs = synth.camera_segments(64, 64, seed=64) if kind == "camera" else synth.bounce_segments(4096, seed=65)
        R = 0.01
    outs = []
    for k, pf in ((1, False), (1, True), (3, False), (3, True), (4, False), (4, True), (0, False), (0, True)):
        with bre.BeamGather(0, counters=True, kernel=k, prefilter=pf) as g:
            g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
            outs.append(g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=R, counts=True))
    assert np.array_equal(outs[0]["seg_rgb"], outs[1]["seg_rgb"])
    assert np.array_equal(outs[0]["counts"], outs[1]["counts"])
    # kernel 3 visits beams in a different order: same sets, sums equal to rounding
    for o in outs[2:]:
        assert np.array_equal(outs[0]["counts"], o["counts"])
        assert _seg_close(o["seg_rgb"], outs[0]["seg_rgb"]) <= SEG_RTOL
    assert np.array_equal(outs[2]["seg_rgb"], outs[3]["seg_rgb"])
    assert np.array_equal(outs[4]["seg_rgb"], outs[5]["seg_rgb"])
    assert np.array_equal(outs[6]["seg_rgb"], outs[7]["seg_rgb"])


@pytest.mark.parametrize("offset", [0.0, 37.5, -250.0])
def test_prefilters_at_the_threshold(bre, oracle, offset):
    """Beams whose line passes at distance (R + r)(1 + e) of a segment, e in [-1e-3, 1e-3], at
    coordinates far from the origin: the packet bundle test and the separable per-lane prefilter
    may only drop pairs the reference computes as d >= R + r (exact contribution sets)."""
    rng = np.random.default_rng(int(abs(offset)) + 3)
    R, r = np.float32(0.02), np.float32(0.01)
    n = 4096
    base = np.float32(offset) + rng.random((n, 3), np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    seg_len = np.float32(0.5)
    o = base.astype(np.float32)
    p = (o + d * seg_len).astype(np.float32)
    # beam: direction e perpendicular to d, through a point at distance (R + r)(1 + eps) from the
    # segment's midpoint along a third direction perpendicular to both
    e = np.cross(d, rng.normal(size=(n, 3))).astype(np.float32)
    e /= np.linalg.norm(e, axis=1, keepdims=True)
    f = np.cross(d, e).astype(np.float32)
    eps = rng.uniform(-1e-3, 1e-3, n).astype(np.float32)
    mid = (o + d * (seg_len / 2)).astype(np.float32)
    c = (mid + f * ((R + r) * (1 + eps))[:, None]).astype(np.float32)
    start = (c - e * np.float32(0.3)).astype(np.float32)
    end = (c + e * np.float32(0.3)).astype(np.float32)
    beams = {"start": start, "end": end, "radius": np.full(n, r, np.float32),
             "power": rng.random((n, 3), np.float32)}
    segs = {"o": o, "p": p, "d": d, "tmax": np.full(n, seg_len, np.float32)}
    ref = oracle.build(beams).gather(segs, float(R))
    assert 0 < ref["contrib"].sum() < ref["cand"].sum()  # both sides of the threshold occur
    for k in (0, 4):
        with bre.BeamGather(0, counters=True, kernel=k) as g:
            g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
            out = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=float(R), counts=True)
        assert np.array_equal(out["counts"][:, 0], ref["cand"]), k
        assert np.array_equal(out["counts"][:, 1], ref["contrib"]), k
        assert _seg_close(out["seg_rgb"], ref["seg_rgb"]) <= SEG_RTOL


@pytest.mark.parametrize("leaf", [16, 64])
def test_kernel4_dense_incoherent_is_deterministic(bre, synth, oracle, leaf):
    """Kernel 4's compaction queue and LDS accumulators on a dense, incoherent set (long beams,
    large radius: many candidates per lane): exact sets, sums to rounding, bit-identical reruns."""
    beams = synth.fog_beams(5000, seed=71, radius=0.03, mean_length=0.7)
    segs = synth.bounce_segments(3000, seed=72)
    ref = oracle.build(beams).gather(segs, 0.04)
    runs = []
    for _ in range(2):
        with bre.BeamGather(0, counters=True, kernel=4, leaf_size=leaf) as g:
            g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
            runs.append(g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=0.04, counts=True))
    assert np.array_equal(runs[0]["counts"][:, 0], ref["cand"])
    assert np.array_equal(runs[0]["counts"][:, 1], ref["contrib"])
    assert _seg_close(runs[0]["seg_rgb"], ref["seg_rgb"]) <= SEG_RTOL
    assert np.array_equal(runs[0]["seg_rgb"], runs[1]["seg_rgb"])


def test_kernel3_rejects_large_leaves(bre, synth):
    beams = synth.fog_beams(500)
    segs = synth.camera_segments(8, 8)
    with bre.BeamGather(0, kernel=3, leaf_size=8) as g:
        g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
        with pytest.raises(bre.BreError):
            g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=0.01)


def test_kernel3_stack_overflow_falls_back_exactly(bre, synth, oracle):
    """Wide incoherent packets over a deep tree can exhaust kernel 3's LDS stack; kernel 1 then
    recomputes on the device and the results stay exact."""
    beams = synth.fog_beams(20000, seed=71, mean_length=0.4)
    segs = synth.camera_segments(48, 32, seed=72)
    ref = oracle.build(beams).gather(segs, 0.01)
    with bre.BeamGather(0, counters=True, kernel=3, split=1, leaf_size=1) as g:
        g.set_option(101, 70)  # internal: 70-entry stack -> most packets overflow
        g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
        out = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=0.01, counts=True)
    assert np.array_equal(out["counts"][:, 0], ref["cand"])
    assert np.array_equal(out["counts"][:, 1], ref["contrib"])
    assert _seg_close(out["seg_rgb"], ref["seg_rgb"]) <= SEG_RTOL



@pytest.mark.parametrize("tile_leaf", [8, 32, 64])
def test_auto_handover_mixed_packets(bre, synth, oracle, tile_leaf):
    """Hand-over mode (kernel 6): coherent camera packets stay in kernel 3, incoherent bounce packets
    go to kernel 4 on the tile tree; one gather over both kinds matches the oracle exactly (sets) and
    to rounding."""
    beams = synth.fog_beams(6000, seed=81, mean_length=0.4)
    cam = synth.camera_segments(32, 32, seed=82)
    bnc = synth.bounce_segments(2048, seed=83, npix=1024)
    segs = {k: np.concatenate([cam[k], bnc[k]]) for k in cam}
    R = 0.012
    ref = oracle.build(beams).gather(segs, R, npix=1024)
    accum = np.zeros((1024, 3), np.float32)
    with bre.BeamGather(0, counters=True, kernel=6) as g:
        g.set_option(bre.OPT_TILE_LEAF, tile_leaf)
        g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
        out = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], segs["pixel"], R=R, npix=1024, accum=accum,
                       counts=True)
        st = g.stats()
    assert st["redo_items"] > 0  # the bounce packets were handed over
    assert np.array_equal(out["counts"][:, 0], ref["cand"])
    assert np.array_equal(out["counts"][:, 1], ref["contrib"])
    assert _seg_close(out["seg_rgb"], ref["seg_rgb"]) <= SEG_RTOL
    assert _rel_l2(accum, ref["accum"]) <= 1e-6


@pytest.mark.parametrize("leaf", [16, 32])
def test_kernel4_leaf_orders_are_bit_identical(bre, synth, oracle, leaf):
    """Kernel 4's prefilter-first leaf scan (tile_mode 1, default) and box-first scan (0) queue the
    contributing pairs in the same (leaf, beam, lane) order: same counts, bit-identical sums, and
    both exact against the oracle (including axis-parallel rays, which take the slab test)."""
    beams = synth.fog_beams(6000, seed=81, radius=0.03, mean_length=0.6)
    segs = synth.bounce_segments(2500, seed=82)
    segs["d"][::97] = np.array([0.0, 0.0, 1.0], np.float32)  # axis-parallel rays (infinite 1/d)
    segs["p"][::97] = segs["o"][::97] + segs["tmax"][::97, None] * segs["d"][::97]
    ref = oracle.build(beams).gather(segs, 0.04)
    outs = []
    for mode in (0, 1):
        with bre.BeamGather(0, counters=True, kernel=4, leaf_size=leaf) as g:
            g.set_option(104, mode)
            g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
            outs.append(g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=0.04, counts=True))
    for o in outs:
        assert np.array_equal(o["counts"][:, 0], ref["cand"])
        assert np.array_equal(o["counts"][:, 1], ref["contrib"])
        assert _seg_close(o["seg_rgb"], ref["seg_rgb"]) <= SEG_RTOL
    assert np.array_equal(outs[0]["seg_rgb"], outs[1]["seg_rgb"])
