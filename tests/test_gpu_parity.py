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


KERNELS = [0, 2, 4]


def _production_counts(bre, beams, segs, R, **kw):
    """The production configuration (kernel 0, counters OFF: the timed instantiation), with the
    contributions counted by its own control flow."""
    with bre.BeamGather(0, counters=False, kernel=0, **kw) as g:
        g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
        return g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=R, counts=True)


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("leaf", [1, 4, 8, 64])
def test_camera_segments_match_oracle(bre, synth, oracle, kernel, leaf):
    beams = synth.fog_beams(3000, seed=12345)
    segs = synth.camera_segments(48, 40, seed=777)
    R = 0.01
    ref = oracle.build(beams).gather(segs, R)
    with bre.BeamGather(0, counters=True, kernel=kernel, leaf_size=leaf) as g:
        if kernel == 0:
            g.set_option(bre.OPT_TILE_LEAF, leaf)
        g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
        out = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], segs["pixel"], R=R, counts=True)
        st = g.stats()
    assert np.array_equal(out["counts"][:, 0], ref["cand"]), "candidate sets differ"
    assert np.array_equal(out["counts"][:, 1], ref["contrib"]), "contribution sets differ"
    assert _seg_close(out["seg_rgb"], ref["seg_rgb"]) <= SEG_RTOL
    assert st["candidates"] == int(ref["cand"].sum())
    assert st["contributions"] == int(ref["contrib"].sum())


@pytest.mark.parametrize("kernel", KERNELS)
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
        for k in KERNELS:
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


@pytest.mark.parametrize("kernel", [0, 4])
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
    """The conservative line-distance rejects must not drop any contributing pair: outputs with and
    without them are bit-identical (same queue order), on coherent, incoherent and long-beam /
    large-radius inputs, for the counting and the production instantiations."""
    if kind == "long":
        beams = synth.fog_beams(6000, seed=61, radius=0.05, mean_length=0.8)
        segs = synth.bounce_segments(6000, seed=62)
        R = 0.08
    else:
        beams = synth.fog_beams(20000, seed=63)
        segs = synth.camera_segments(64, 64, seed=64) if kind == "camera" else synth.bounce_segments(4096, seed=65)
        R = 0.01
    outs = {}
    for counters in (True, False):
        for pf in (False, True):
            with bre.BeamGather(0, counters=counters, kernel=0, prefilter=pf) as g:
                g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
                outs[counters, pf] = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=R, counts=True)
    ref = outs[True, True]
    for key, o in outs.items():
        assert np.array_equal(o["seg_rgb"], ref["seg_rgb"]), key
        assert np.array_equal(o["counts"][:, 1], ref["counts"][:, 1]), key
    assert np.array_equal(outs[True, False]["counts"], ref["counts"])


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
    prod = _production_counts(bre, beams, segs, float(R))
    assert np.array_equal(prod["counts"][:, 1], ref["contrib"])
    assert _seg_close(prod["seg_rgb"], ref["seg_rgb"]) <= SEG_RTOL


@pytest.mark.parametrize("kind", ["threshold", "dense", "axis"])
def test_production_kernel_pair_exact(bre, synth, oracle, kind):
    """The timed instantiation (kernel 0, counters off) per segment against the oracle: exact
    contribution counts through its own control flow, sums to rounding, and bit-identical to the
    counting instantiation (same queue order)."""
    rng = np.random.default_rng(7)
    if kind == "dense":
        beams = synth.fog_beams(5000, seed=71, radius=0.03, mean_length=0.7)
        segs = synth.bounce_segments(3000, seed=72)
        R = 0.04
    elif kind == "axis":
        beams = synth.fog_beams(6000, seed=81, radius=0.03, mean_length=0.6)
        segs = synth.bounce_segments(2500, seed=82)
        segs["d"][::97] = np.array([0.0, 0.0, 1.0], np.float32)  # axis-parallel rays (infinite 1/d)
        segs["p"][::97] = segs["o"][::97] + segs["tmax"][::97, None] * segs["d"][::97]
        R = 0.04
    else:
        n = 3000
        Rf, r = np.float32(0.02), np.float32(0.01)
        o = rng.random((n, 3), np.float32)
        d = rng.normal(size=(n, 3)).astype(np.float32)
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        p = (o + d * np.float32(0.5)).astype(np.float32)
        e = np.cross(d, rng.normal(size=(n, 3))).astype(np.float32)
        e /= np.linalg.norm(e, axis=1, keepdims=True)
        f = np.cross(d, e).astype(np.float32)
        eps = rng.uniform(-1e-3, 1e-3, n).astype(np.float32)
        c = (o + d * np.float32(0.25) + f * ((Rf + r) * (1 + eps))[:, None]).astype(np.float32)
        beams = {"start": (c - e * np.float32(0.3)).astype(np.float32), "end": (c + e * np.float32(0.3)).astype(np.float32),
                 "radius": np.full(n, r, np.float32), "power": rng.random((n, 3), np.float32)}
        segs = {"o": o, "p": p, "d": d, "tmax": np.full(n, 0.5, np.float32)}
        R = float(Rf)
    ref = oracle.build(beams).gather(segs, R)
    prod = _production_counts(bre, beams, segs, R)
    assert (prod["counts"][:, 0] == -1).all()
    assert np.array_equal(prod["counts"][:, 1], ref["contrib"])
    assert _seg_close(prod["seg_rgb"], ref["seg_rgb"]) <= SEG_RTOL
    with bre.BeamGather(0, counters=True, kernel=0) as g:
        g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
        cnt = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=R, counts=True)
    assert np.array_equal(cnt["counts"][:, 0], ref["cand"])
    assert np.array_equal(cnt["seg_rgb"], prod["seg_rgb"])


@pytest.mark.parametrize("kernel", [0, 2])
def test_stack_overflow_is_an_error_without_counters(bre, synth, kernel):
    """A traversal-stack overflow drops contributions: it must surface as BRE_ERR_STATE at the next
    synchronising call with the default options (counters off), and the context stays usable."""
    beams = synth.fog_beams(20000, seed=71, mean_length=0.4)
    segs = synth.camera_segments(48, 32, seed=72)
    with bre.BeamGather(0, kernel=kernel, split=1) as g:
        g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
        g.set_option(101, 2)  # internal: a 2-entry traversal stack
        with pytest.raises(bre.BreError) as ei:
            g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=0.01)
        assert ei.value.status == 4  # BRE_ERR_STATE
        g.set_option(101, 0)
        out = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=0.01)  # sticky flag was cleared
        assert out["seg_rgb"].any()


def test_device_pixel_error_reported_at_synchronize(bre, synth):
    """bre_gather_device is asynchronous: a bad seg_pixel is reported by the next synchronising call."""
    import torch

    beams = synth.fog_beams(3000, seed=5)
    segs = synth.camera_segments(16, 16, seed=6)
    segs["pixel"][7] = 10_000
    dseg = {k: torch.from_numpy(v).cuda().contiguous() for k, v in segs.items()}
    with bre.BeamGather(0) as g:
        g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
        acc = torch.zeros((256, 3), dtype=torch.float32, device="cuda")
        g.gather_device(dseg["o"], dseg["p"], dseg["d"], dseg["tmax"], dseg["pixel"], 0.01, 256, accum=acc)
        with pytest.raises(bre.BreError) as ei:
            g.synchronize()
        assert ei.value.status == 1  # BRE_ERR_INVALID_ARG
        g.synchronize()  # cleared


@pytest.mark.parametrize("kind", ["camera", "bounce", "long"])
def test_transposed_scan_is_bit_identical(bre, synth, kind):
    """The transposed scan (one on-lane segment per step against all beams of a tile) queues each
    segment's pairs in the same beam order as the beam-major scan, so forcing it everywhere (threshold
    64: whenever fewer lanes are on than 8x the kept beams) or never (0) changes no output bit; the
    default (6) mixes both within one gather."""
    if kind == "long":
        beams = synth.fog_beams(6000, seed=81, radius=0.05, mean_length=0.8)
        segs = synth.bounce_segments(6000, seed=82)
        R = 0.08
    else:
        beams = synth.fog_beams(20000, seed=83)
        segs = synth.camera_segments(64, 64, seed=84) if kind == "camera" else synth.bounce_segments(4096, seed=85)
        R = 0.01
    outs = {}
    for t in (0, 6, 64):
        with bre.BeamGather(0, counters=False, kernel=0) as g:
            g.set_option(108, t)
            g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
            outs[t] = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=R, counts=True)
    assert outs[0]["counts"][:, 1].sum() > 0
    for t in (6, 64):
        assert np.array_equal(outs[t]["seg_rgb"], outs[0]["seg_rgb"]), t
        assert np.array_equal(outs[t]["counts"][:, 1], outs[0]["counts"][:, 1]), t


def test_transposed_scan_skips_packet_rejected_parallel_beams(bre, oracle):
    """a beam the packet rejects is staged with thr_sq = -inf, but scan_keep_mask only
    rejects when u >= 0.0101, so a rejected beam nearly parallel to the segments would get a keep bit
    in the transposed scan (lane = beam) unless the push is masked with the packet's kept beams.  One
    leaf tile holds 24 beams crossing a packet of 64 parallel segments and 40 beams parallel to them
    but far away (packet box reject).  The production kernel's own queue length (counted whenever
    per-segment counts are asked for) must be the same with the transposed scan forced on (threshold
    64) and off (0), and so must every output bit."""
    rng = np.random.default_rng(5)
    n_seg = 64
    o = np.stack([np.full(n_seg, 0.1), np.linspace(0.10, 0.20, n_seg), np.full(n_seg, 0.5)], 1).astype(np.float32)
    d = np.tile(np.array([1.0, 0.0, 0.0], np.float32), (n_seg, 1))
    segs = {"o": o, "p": (o + d * np.float32(0.8)).astype(np.float32), "d": d,
            "tmax": np.full(n_seg, 0.8, np.float32)}
    xs = rng.uniform(0.15, 0.85, 24).astype(np.float32)
    cross_s = np.stack([xs, np.full(24, 0.15), np.full(24, 0.2)], 1).astype(np.float32)
    cross_e = np.stack([xs, np.full(24, 0.15), np.full(24, 0.8)], 1).astype(np.float32)
    y = rng.uniform(0.80, 0.90, 40).astype(np.float32)
    par_s = np.stack([np.full(40, 0.1), y, np.full(40, 0.5)], 1).astype(np.float32)
    par_e = np.stack([np.full(40, 0.9), y + np.float32(1e-3), np.full(40, 0.5)], 1).astype(np.float32)
    beams = {"start": np.concatenate([cross_s, par_s]), "end": np.concatenate([cross_e, par_e]),
             "radius": np.full(64, 0.01, np.float32), "power": rng.random((64, 3), np.float32)}
    R = 0.02
    ref = oracle.build(beams).gather(segs, R)
    assert ref["contrib"].sum() > 0
    outs, queued = {}, {}
    for t in (0, 64):
        with bre.BeamGather(0, counters=False, timing=True, kernel=0) as g:
            g.set_option(108, t)
            g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
            outs[t] = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=R, counts=True)
            queued[t] = g.stats()["queued_pairs"]
    assert np.array_equal(outs[64]["counts"][:, 1], ref["contrib"])
    assert queued[0] > 0
    assert queued[64] == queued[0], queued
    assert np.array_equal(outs[64]["seg_rgb"], outs[0]["seg_rgb"])


def test_removed_kernels_are_rejected(bre):
    with bre.BeamGather(0) as g:
        for k in (1, 3, 6, 7):
            with pytest.raises(bre.BreError):
                g.set_option(bre.OPT_KERNEL, k)


@pytest.mark.parametrize("leaf", [16, 64])
def test_kernel4_dense_incoherent_is_deterministic(bre, synth, oracle, leaf):
    """The tile kernel's compaction queue and LDS accumulators on a dense, incoherent set (long
    beams, large radius: many candidates per lane): exact sets, sums to rounding, bit-identical reruns."""
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


def test_segment_repeated_through_whole_batches(bre, oracle):
    """A few segments, each crossed by ~1500 beams: the exact-stage batches hold up to 64 pairs of one
    segment, so its accumulation runs all its read-modify-write rounds (ranks 0-7) and adds ranks
    >= 8 by LDS atomics; the beam-major (tscan 0) and transposed (6) scans queue them alike.  Exact
    contribution counts and sums to rounding against the oracle, bit-identical across the scans."""
    rng = np.random.default_rng(11)
    Rf, r = np.float32(0.02), np.float32(0.01)
    axes = [(np.array([0.5, 0.5, 0.1], np.float32), np.array([0.0, 0.0, 1.0], np.float32)),
            (np.array([0.2, 0.7, 0.3], np.float32), np.array([1.0, 0.0, 0.0], np.float32)),
            (np.array([0.3, 0.1, 0.6], np.float32), np.array([0.0, 1.0, 0.0], np.float32))]
    starts, ends = [], []
    for o, d in axes:
        m = 1500
        c = o + d * rng.uniform(0.05, 0.75, m).astype(np.float32)[:, None]
        e = np.cross(d, rng.normal(size=(m, 3))).astype(np.float32)
        e /= np.linalg.norm(e, axis=1, keepdims=True)
        c = (c + np.cross(d, e) * ((Rf + r) * rng.uniform(-0.5, 0.5, m)).astype(np.float32)[:, None]).astype(np.float32)
        starts.append(c - e * np.float32(0.3))
        ends.append(c + e * np.float32(0.3))
    start, end = np.concatenate(starts).astype(np.float32), np.concatenate(ends).astype(np.float32)
    beams = {"start": start, "end": end, "radius": np.full(len(start), r, np.float32),
             "power": rng.random((len(start), 3), np.float32)}
    o = np.stack([a[0] for a in axes]).astype(np.float32)
    d = np.stack([a[1] for a in axes]).astype(np.float32)
    segs = {"o": o, "p": (o + d * np.float32(0.8)).astype(np.float32), "d": d, "tmax": np.full(3, 0.8, np.float32)}
    ref = oracle.build(beams).gather(segs, float(Rf))
    assert ref["contrib"].min() > 500
    outs = {}
    for t in (0, 6):
        with bre.BeamGather(0, counters=False, kernel=0) as g:
            g.set_option(108, t)
            g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
            outs[t] = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=float(Rf), counts=True)
    out = outs[6]
    assert np.array_equal(out["counts"][:, 1], ref["contrib"])
    assert _seg_close(out["seg_rgb"], ref["seg_rgb"]) <= SEG_RTOL
    assert np.array_equal(out["seg_rgb"], outs[0]["seg_rgb"])


@pytest.mark.parametrize("beam_key", [0, 1, 2])
def test_tree_and_segment_orders_give_exact_sets(bre, synth, oracle, beam_key):
    """The tree order (option 110: centroid Morton 0, (start, end) Morton 1, (start, end) Hilbert 2 =
    default) and the segment coherence-sort key (option 105: 0-4, Hilbert 4 = default) only reorder
    work: every combination gives the oracle's exact contribution counts and its sums to rounding;
    out-of-range keys are rejected."""
    beams = synth.fog_beams(20000, seed=91)
    segs = synth.bounce_segments(4096, seed=92)
    ref = oracle.build(beams).gather(segs, 0.01)
    assert ref["contrib"].sum() > 0
    for sort_key in range(5):
        with bre.BeamGather(0, counters=False, kernel=0) as g:
            g.set_option(110, beam_key)
            g.set_option(105, sort_key)
            g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
            out = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=0.01, counts=True)
        assert np.array_equal(out["counts"][:, 1], ref["contrib"]), sort_key
        assert _seg_close(out["seg_rgb"], ref["seg_rgb"]) <= SEG_RTOL, sort_key
    with bre.BeamGather(0) as g:
        for opt, bad in ((110, 3), (110, -1), (105, 5)):
            with pytest.raises(bre.BreError):
                g.set_option(opt, bad)
