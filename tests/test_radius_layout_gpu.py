"""Beam sets with and without one common radius give the reference's per-segment results.

The build checks whether every valid beam has the same radius (k_prep: min / max of the radius bits).
If so, the 64-B BeamRec carries the beam's scaled power in place of (radius, pad) and every kernel
reads the radius from the set (BeamSet); otherwise the record keeps its radius and the power comes
from its own array (bre_device.h BeamRec).  The integrator's beams always share the pass radius
(photonbeam.cpp:292), so the other tests run the uniform layout; these run mixed radii (one outlier
beam, and radii drawn per beam) through every kernel against the oracle, and check that the two
layouts give bit-identical sums on the same uniform set (the uniform layout also divides by the
shared MaxDistance through its reciprocal, bre_math.h div_by_shared)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEG_RTOL = 1e-5


def _seg_close(gpu, ref):
    scale = np.maximum(np.abs(ref).max(axis=1, keepdims=True), 1e-30)
    return (np.abs(gpu - ref) / scale).max()


def _mixed(synth, kind):
    beams = synth.fog_beams(4000, seed=31, radius=0.012, mean_length=0.4)
    if kind == "outlier":
        beams["radius"][1717] = np.float32(0.03)
    else:
        rng = np.random.default_rng(32)
        beams["radius"] = rng.uniform(0.004, 0.03, beams["radius"].shape[0]).astype(np.float32)
    return beams


@pytest.mark.parametrize("kind", ["outlier", "random"])
@pytest.mark.parametrize("kernel", [0, 2, 4, 5])
def test_mixed_radii_match_oracle(bre, synth, oracle, kind, kernel):
    beams = _mixed(synth, kind)
    segs = synth.bounce_segments(3000, seed=33)
    R = 0.015
    ref = oracle.build(beams).gather(segs, R)
    with bre.BeamGather(0, counters=True, kernel=kernel) as g:
        g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
        out = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=R, counts=True)
    if kernel != 5:  # kernel 5 enumerates chunks, not the reference's candidates
        assert np.array_equal(out["counts"][:, 0], ref["cand"])
    assert np.array_equal(out["counts"][:, 1], ref["contrib"])
    assert _seg_close(out["seg_rgb"], ref["seg_rgb"]) <= SEG_RTOL


@pytest.mark.parametrize("kind", ["outlier", "random"])
def test_mixed_radii_production_kernel(bre, synth, oracle, kind):
    """The timed instantiation (kernel 0, counters off) on mixed radii."""
    beams = _mixed(synth, kind)
    segs = synth.bounce_segments(3000, seed=34)
    R = 0.015
    ref = oracle.build(beams).gather(segs, R)
    with bre.BeamGather(0, counters=False, kernel=0) as g:
        g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
        out = g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=R, counts=True)
    assert np.array_equal(out["counts"][:, 1], ref["contrib"])
    assert _seg_close(out["seg_rgb"], ref["seg_rgb"]) <= SEG_RTOL


def test_uniform_and_split_layouts_bit_identical(bre, synth):
    """One uniform set gathered with the power in the records (default) and with the split layout
    (internal option 113): the same tree and queue order, so the per-segment sums and counts are
    bit-identical -- the layout changes where values are read, not what."""
    beams = synth.fog_beams(3000, seed=35, radius=0.01, mean_length=0.5)
    segs = synth.bounce_segments(2500, seed=36)
    R = 0.012
    res = []
    for split in (0, 1):
        with bre.BeamGather(0, counters=False, kernel=0) as g:
            g.set_option(113, split)
            g.set_beams(beams["start"], beams["end"], beams["radius"], beams["power"])
            res.append(g.gather(segs["o"], segs["p"], segs["d"], segs["tmax"], R=R, counts=True))
    assert res[0]["counts"][:, 1].sum() > 1000
    assert np.array_equal(res[0]["counts"], res[1]["counts"])
    assert np.array_equal(res[0]["seg_rgb"].view(np.uint32), res[1]["seg_rgb"].view(np.uint32))


@pytest.mark.parametrize("iteration", [0, 12])
def test_layouts_bit_identical_on_c2(bre, scene_mod_gpu, iteration):
    """The same on real C2 data (millions of contributing pairs): the uniform layout also divides by
    the set's MaxDistance through its reciprocal (bre_math.h div_by_shared), which must give the
    correctly rounded quotient of every pair, as the split layout's division does."""
    import torch

    scene = scene_mod_gpu.cornell_scene(0.05, 0.5, 0.0)
    R = bre.beam_radius_at(0.01, 0.5, iteration)
    out = {}
    for split in (0, 1):
        with bre.BeamGather(0) as g:
            g.set_option(113, split)
            g.trace_photons(scene, 300_000, iteration, 5, R)
            n = g.camera_pass(scene, 256, 256, iteration, 5, True, True)
            rgb = torch.zeros((n, 3), dtype=torch.float32, device="cuda")
            cnt = torch.zeros((n, 2), dtype=torch.int32, device="cuda")
            g.gather_camera_segments(R, seg_rgb=rgb, counts=cnt)
            g.synchronize()
            out[split] = (rgb.cpu().numpy(), cnt.cpu().numpy())
    assert out[0][1][:, 1].sum() > 1_000_000
    assert np.array_equal(out[0][1], out[1][1])
    assert np.array_equal(out[0][0].view(np.uint32), out[1][0].view(np.uint32))
