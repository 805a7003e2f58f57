"""The TIMED configuration on REAL C2 data, segment by segment ("next round" item 1).

C2 = BASELINE.json configs[1]: Cornell box + homogeneous fog, 512x512, 1M photons per iteration,
maxdepth 5, R0 0.01, alpha 0.5.  For iterations 0 and 15 the photon pass, BVH build, camera pass,
coherence sort and gather run exactly as bench.py times them (kernel 0, counters OFF, segment sort
on); bre_gather_camera_segments only scatters the per-segment sums and the contribution counts
(counted by the production instantiation's own control flow) back to camera-pass order.  ~1,000
randomly sampled segments are then gathered by the oracle (reference SAH tree over the FULL beam
set, photonbeam.cpp:494-508) and compared: contribution counts exactly, per-segment RGB within the
float32 summation-order bound max(1e-5, 4 u sqrt(n)) relative (n contributions, u = 2^-24).  The pixel sums are also checked against the per-segment
sums (the scatter and the production accumulation agree)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W = H = 512
PHOTONS = 1_000_000
NSAMPLE = 1000


@pytest.mark.parametrize("iteration", [0, 15])
def test_c2_production_gather_matches_oracle_per_segment(bre, oracle, scene_mod_gpu, iteration):
    import torch

    sc = scene_mod_gpu
    scene = sc.cornell_scene(0.05, 0.5, 0.0)
    R = bre.beam_radius_at(0.01, 0.5, iteration)
    with bre.BeamGather(0) as g:  # the bench's configuration: kernel 0, counters off, sort on
        nb = g.trace_photons(scene, PHOTONS, iteration, 5, R)
        n = g.camera_pass(scene, W, H, iteration, 5, True, True)
        seg_rgb = torch.zeros((n, 3), dtype=torch.float32, device="cuda")
        counts = torch.zeros((n, 2), dtype=torch.int32, device="cuda")
        ld = torch.zeros((W * H, 3), dtype=torch.float32, device="cuda")
        g.gather_camera_segments(R, accum=ld, seg_rgb=seg_rgb, counts=counts)
        g.synchronize()
        beams = g.get_beams()
        segs = g.get_segments()
    seg_rgb = seg_rgb.cpu().numpy()
    counts = counts.cpu().numpy()
    ld = ld.cpu().numpy()
    assert nb > 2_000_000 and n > 500_000
    assert (counts[:, 0] == -1).all()
    # the production accumulation equals the per-segment sums added by pixel
    acc = np.zeros((W * H, 3), np.float64)
    np.add.at(acc, segs["pixel"], seg_rgb.astype(np.float64))
    assert np.abs(ld - acc).max() <= 1e-5 * max(float(np.abs(acc).max()), 1e-30)
    # oracle on a seeded sample of the same segments against all beams
    idx = np.random.default_rng(1000 + iteration).choice(n, NSAMPLE, replace=False)
    sample = {k: np.ascontiguousarray(segs[k][idx]) for k in ("o", "p", "d", "tmax", "pixel")}
    bvh = oracle.build(beams)
    ref = bvh.gather(sample, R, nthreads=16, chunk=8)
    bvh.close()
    assert ref["contrib"].sum() > 1_000_000  # dense real data (~49k contributions per segment at C2)
    assert np.array_equal(counts[idx, 1], ref["contrib"]), "production contribution counts differ"
    # per-segment tolerance: both sides are float32 sums of the same n positive terms in different
    # orders; each sum's rounding error has a std of ~u sqrt(n) / 3 relative (u = 2^-24), so the
    # difference is held to 4 u sqrt(n) (~8.5 sigma; 5.3e-5 at C2's ~49k terms), floor 1e-5
    scale = np.maximum(np.abs(ref["seg_rgb"]).max(axis=1), 1e-30)
    err = np.abs(seg_rgb[idx] - ref["seg_rgb"]).max(axis=1) / scale
    tol = np.maximum(1e-5, 4 * 2.0 ** -24 * np.sqrt(ref["contrib"].astype(np.float64)))
    worst = int(np.argmax(err / tol))
    assert (err <= tol).all(), (float(err[worst]), float(tol[worst]), int(ref["contrib"][worst]))
