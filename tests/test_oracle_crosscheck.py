"""The C++ oracle against the independent Python restatement (tests/refpy.py), bit for bit, and the
oracle's SAH-tree gather against its BVH-free brute force (same candidate set, by construction of
the reference: SURVEY.md §7 "key enabler")."""
import numpy as np
import pytest

import refpy


@pytest.fixture(scope="module")
def rng():
    return np.random.default_rng(20251015)


def test_world_bound_bitwise(oracle, rng):
    n = 400
    start = rng.random((n, 3), dtype=np.float32)
    end = (start + rng.normal(size=(n, 3)).astype(np.float32) * np.float32(0.3)).astype(np.float32)
    radius = (rng.random(n, dtype=np.float32) * np.float32(0.05)).astype(np.float32)
    box = oracle.beam_bounds(start, end, radius)
    for i in range(n):
        lo, hi = refpy.world_bound(start[i], end[i], radius[i])
        assert np.array_equal(np.array(lo + hi, np.float32), box[i]), i


def test_closest_points_bitwise(oracle, rng):
    for i in range(600):
        pts = rng.random((4, 3), dtype=np.float32)
        if i % 7 == 0:
            pts[1] = pts[0]  # zero-length segment
        if i % 11 == 0:
            pts[3] = pts[2] + (pts[1] - pts[0]) * np.float32(0.5)  # near-parallel
        ok, ac, bc = oracle.closest_points(*pts)
        ok2, ac2, bc2 = refpy.closest_points(*pts)
        assert ok == ok2, i
        if ok:
            assert np.array_equal(ac, np.array(ac2, np.float32)), i
            assert np.array_equal(bc, np.array(bc2, np.float32)), i


def test_intersect_p_bitwise(oracle, rng):
    for i in range(1500):
        lo = rng.random(3, dtype=np.float32)
        hi = (lo + rng.random(3, dtype=np.float32) * np.float32(0.3)).astype(np.float32)
        o = (rng.random(3, dtype=np.float32) * np.float32(1.4) - np.float32(0.2)).astype(np.float32)
        d = rng.normal(size=3).astype(np.float32)
        if i % 5 == 0:
            d[i % 3] = 0.0
        if i % 13 == 0:
            o[0] = lo[0]  # origin on a slab plane (0 * inf = NaN path)
        tmax = np.float32(rng.random() * 2)
        got = oracle.intersect_box(np.concatenate([lo, hi]), o, d, tmax)
        assert got == refpy.intersect_p(lo, hi, o, d, tmax), i


def test_contributions_bitwise_small_scene(oracle, synth):
    beams = synth.fog_beams(60, seed=5, mean_length=0.5)
    segs = synth.bounce_segments(60, seed=6)
    R = 0.03
    bf = oracle.bruteforce(beams, segs, R)
    for s in range(60):
        acc = [np.float32(0)] * 3
        cand = 0
        for b in range(60):
            lo, hi = refpy.world_bound(beams["start"][b], beams["end"][b], beams["radius"][b])
            if not refpy.intersect_p(lo, hi, segs["o"][s], segs["d"][s], segs["tmax"][s]):
                continue
            cand += 1
            c = refpy.contribution((beams["start"][b], beams["end"][b], beams["radius"][b], beams["power"][b]),
                                   segs["o"][s], segs["p"][s], R)
            if c is not None:
                acc = [acc[k] + c[k] for k in range(3)]
        assert cand == bf["cand"][s]
        assert np.array_equal(np.array(acc, np.float32), bf["seg_rgb"][s]), s


@pytest.mark.parametrize("kind", ["camera", "bounce"])
def test_sah_tree_equals_bruteforce(oracle, synth, kind):
    beams = synth.fog_beams(1500, seed=77)
    segs = synth.camera_segments(40, 30, seed=78) if kind == "camera" else synth.bounce_segments(1200, seed=79)
    R = 0.01
    tree = oracle.build(beams).gather(segs, R)
    bf = oracle.bruteforce(beams, segs, R)
    assert np.array_equal(tree["cand"], bf["cand"])
    assert np.array_equal(tree["contrib"], bf["contrib"])
    scale = np.maximum(np.abs(bf["seg_rgb"]).max(axis=1, keepdims=True), 1e-30)
    assert (np.abs(tree["seg_rgb"] - bf["seg_rgb"]) / scale).max() <= 1e-5


def test_sah_tree_shape_invariants(oracle, synth):
    beams = synth.fog_beams(999, seed=3)
    bvh = oracle.build(beams)
    assert bvh.node_count() == 2 * 999 - 1  # leaf size 1, no duplicate centroids
    assert bvh.max_leaf() == 1


def test_multithreaded_gather_equals_serial(oracle, synth):
    beams = synth.fog_beams(3000, seed=1)
    segs = synth.camera_segments(32, 32, seed=2)
    bvh = oracle.build(beams)
    a = bvh.gather(segs, 0.01, nthreads=1)
    b = bvh.gather(segs, 0.01, nthreads=4, chunk=16)
    for k in ("seg_rgb", "cand", "visit", "contrib"):
        assert np.array_equal(a[k], b[k])


@pytest.mark.parametrize("kind", ["camera", "bounce"])
def test_skip_gather_equals_reference_form(oracle, synth, kind):
    """The image-parity gather (ora_gather_skip) skips only candidates whose double line distance
    proves they cannot contribute: its per-segment sums and counts are the reference form's bit for
    bit, and it does skip (most candidates, at a small radius)."""
    beams = synth.fog_beams(4000, seed=81)
    segs = synth.camera_segments(40, 30, seed=82) if kind == "camera" else synth.bounce_segments(1200, seed=83)
    bvh = oracle.build(beams)
    for R in (0.002, 0.01, 0.05):
        ref = bvh.gather(segs, R, nthreads=2)
        got = bvh.gather_skip(segs, R, npix=int(segs["pixel"].max()) + 1, nthreads=3)
        assert np.array_equal(ref["seg_rgb"].view(np.uint32), got["seg_rgb"].view(np.uint32))
        assert np.array_equal(ref["cand"], got["cand"]) and np.array_equal(ref["contrib"], got["contrib"])
        assert got["skipped"].sum() > 0.5 * (got["cand"].sum() - got["contrib"].sum())
        # the film: per-segment sums added in segment order
        acc = np.zeros_like(got["accum"])
        for s in range(segs["tmax"].shape[0]):
            acc[segs["pixel"][s]] += got["seg_rgb"][s]
        assert np.array_equal(acc, got["accum"])
