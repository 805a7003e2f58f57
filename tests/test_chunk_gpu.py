"""Kernel 5 (capsule-chunk index, csrc/bre_chunk.hip) against the CPU oracle.

Kernel 5 never enumerates the reference's non-contributing box hits, so its per-segment count
seg_counts[0] is not the reference's candidate count C.  What it must reproduce exactly is the
SET of contributing pairs (d < R + r AND the reference's box test on the group box): per-segment
contribution counts are compared EXACTLY with the oracle's (SAH tree, reference arithmetic), and
per-segment RGB within 1e-5 relative (summation order only; each pair is bit-identical).
Cases cover the quirks the index must not lose: beam-LINE contributions whose closest beam point
lies outside the beam (ComputeClosestPoints keeps t1 unclamped when t0 is inside the segment,
photonbeam.cpp:178-181), the signed-direction box that shrinks (photonbeambvh.h:60-72), equal
centroids sharing a group box, axis-parallel rays (1/d infinite) and zero-length segments.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEG_RTOL = 1e-5


def _seg_err(gpu, ref):
    scale = np.maximum(np.abs(ref).max(axis=1, keepdims=True), 1e-30)
    return float((np.abs(gpu - ref) / scale).max())


def _run(bre, beams, segs, R, npix=0, **opt):
    with bre.BeamGather(0, counters=True, kernel=5) as g:
        for k, v in opt.items():
            g.set_option(getattr(bre, "OPT_" + k.upper()), v)
        g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
        out = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], segs.get("pixel"), R=R, counts=True)
        st = g.stats()
    return out, st


@pytest.mark.parametrize("chunk_len,leaf", [(400, 1), (150, 1), (1200, 4)])
def test_chunk_camera_segments_match_oracle(bre, synth, oracle, chunk_len, leaf):
    beams = synth.fog_beams(3000, seed=12345)
    segs = synth.camera_segments(48, 40, seed=777)
    R = 0.01
    ref = oracle.build(beams).gather(segs, R)
    out, st = _run(bre, beams, segs, R, chunk_len=chunk_len, chunk_leaf=leaf)
    assert np.array_equal(out["counts"][:, 1], ref["contrib"]), "contribution sets differ"
    assert _seg_err(out["seg_rgb"], ref["seg_rgb"]) <= SEG_RTOL
    assert st["contributions"] == int(ref["contrib"].sum())
    assert st["n_chunks"] > 3000


def test_chunk_bounce_segments_match_oracle(bre, synth, oracle):
    beams = synth.fog_beams(3000, seed=99)
    segs = synth.bounce_segments(3000, seed=5)
    R = 0.013
    ref = oracle.build(beams).gather(segs, R)
    out, _ = _run(bre, beams, segs, R)
    assert np.array_equal(out["counts"][:, 1], ref["contrib"])
    assert _seg_err(out["seg_rgb"], ref["seg_rgb"]) <= SEG_RTOL


def test_chunk_line_contributions_beyond_the_beam(bre, oracle):
    """Short beams and long segments crossing their LINE well beyond either end: the reference
    counts those pairs (t1 unclamped) whenever the segment's ray also hits the beam's box."""
    rng = np.random.default_rng(3)
    n = 400
    start = rng.uniform(0.3, 0.7, (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    end = (start + 0.05 * d).astype(np.float32)
    beams = {"start": start, "end": end, "radius": np.full(n, 0.02, np.float32),
             "power": rng.random((n, 3)).astype(np.float32)}
    m = 4000
    o = rng.uniform(0, 1, (m, 3)).astype(np.float32)
    tgt = rng.uniform(0, 1, (m, 3)).astype(np.float32)
    dd = tgt - o
    tm = np.linalg.norm(dd, axis=1).astype(np.float32)
    dd = (dd / tm[:, None]).astype(np.float32)
    segs = {"o": o, "d": dd, "tmax": tm, "p": (o + dd * tm[:, None]).astype(np.float32),
            "pixel": np.arange(m, dtype=np.int32)}
    R = 0.03
    ref = oracle.build(beams).gather(segs, R)
    assert ref["contrib"].sum() > 100
    out, _ = _run(bre, beams, segs, R)
    assert np.array_equal(out["counts"][:, 1], ref["contrib"])
    assert _seg_err(out["seg_rgb"], ref["seg_rgb"]) <= SEG_RTOL


def test_chunk_axis_parallel_and_degenerate(bre, synth, oracle):
    beams = synth.fog_beams(1500, seed=21, mean_length=0.4)
    # axis-parallel rays (1/d = inf on two axes) and zero-length segments
    k = 600
    rng = np.random.default_rng(9)
    o = rng.uniform(0.05, 0.95, (k, 3)).astype(np.float32)
    axis = rng.integers(0, 3, k)
    d = np.zeros((k, 3), np.float32)
    d[np.arange(k), axis] = np.where(rng.random(k) < 0.5, 1.0, -1.0)
    tm = rng.uniform(0.0, 0.6, k).astype(np.float32)
    tm[::7] = 0.0
    p = (o + d * tm[:, None]).astype(np.float32)
    segs = {"o": o, "p": p, "d": d, "tmax": tm, "pixel": np.arange(k, dtype=np.int32)}
    R = 0.02
    ref = oracle.build(beams).gather(segs, R)
    out, _ = _run(bre, beams, segs, R)
    assert np.array_equal(out["counts"][:, 1], ref["contrib"])
    assert _seg_err(out["seg_rgb"], ref["seg_rgb"]) <= SEG_RTOL


def test_chunk_group_boxes_and_mirrored_beams(bre, synth, oracle):
    base = synth.fog_beams(400, seed=8, mean_length=0.3)
    start, end = base["start"].copy(), base["end"].copy()
    idx = np.arange(0, 400, 4)
    start2 = np.concatenate([start, end[idx]])
    end2 = np.concatenate([end, start[idx]])
    beams = {"start": start2, "end": end2, "radius": np.full(len(start2), 0.01, np.float32),
             "power": np.concatenate([base["power"], base["power"][idx]])}
    segs = synth.bounce_segments(3000, seed=2)
    R = 0.02
    ref = oracle.build(beams).gather(segs, R)
    out, _ = _run(bre, beams, segs, R)
    assert np.array_equal(out["counts"][:, 1], ref["contrib"])
    assert _seg_err(out["seg_rgb"], ref["seg_rgb"]) <= SEG_RTOL


def test_chunk_matches_kernel0_on_c2_iteration(bre, scene_mod_gpu):
    """A real C2-style iteration (photons and camera paths traced on the GPU, 256k photons,
    128x128): kernel 5 and the reference-enumerating auto kernel give the same contribution count
    per segment and the same image to float summation order."""
    import torch

    sc = scene_mod_gpu
    s = sc.cornell_scene()
    res = {}
    for kern in (0, 5):
        ld = torch.zeros((128 * 128, 3), dtype=torch.float32, device="cuda")
        with bre.BeamGather(0, counters=True, kernel=kern) as g:
            g.trace_photons(s, 250_000, iteration=1, max_depth=5, radius=0.01)
            g.camera_pass(s, 128, 128, iteration=1, max_depth=5, render_surfaces=False)
            seg = g.get_segments()
            out = g.gather(seg["o"], seg["p"], seg["d"], seg["tmax"], seg["pixel"], R=0.01, counts=True)
        res[kern] = out
    assert np.array_equal(res[0]["counts"][:, 1], res[5]["counts"][:, 1])
    assert _seg_err(res[5]["seg_rgb"], res[0]["seg_rgb"]) <= SEG_RTOL


def test_chunk_empty_and_errors(bre, synth):
    segs = synth.camera_segments(8, 8)
    with bre.BeamGather(0, counters=True, kernel=5) as g:
        g.set_beams(np.zeros((0, 3)), np.zeros((0, 3)), np.zeros(0), np.zeros((0, 3)))
        out = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], segs["pixel"], R=0.01, counts=True)
        assert not out["seg_rgb"].any()
        with pytest.raises(bre.BreError):
            g.set_option(bre.OPT_CHUNK_LEN, 1)
        with pytest.raises(bre.BreError):
            g.set_option(bre.OPT_CHUNK_LEAF, 0)
