"""C3 and C5 at their real sizes on the GPU ("next round" item 3).

C3 = BASELINE.json configs[2]: the Cornell box filled with a 64^3 GridDensityMedium of seeded
value-noise smoke (sigma_a 0.5, sigma_s 4.5, Henyey-Greenstein g 0.7), 1024x1024, 5M photons,
iteration 0 (R 0.01): ~11.5M beams, ~257k contributions per estimate.
C5 = configs[4]: the same smoke with 50M photons per pass, progressive radius; its last pass
(iteration 9 of 10, the smallest radius R_9 = R_0 prod (i + 0.5) / (i + 1), photonbeam.cpp:354-356, 562).

For each, the production gather (kernel 0, counters off, coherence sort on -- the bench
configuration) of every camera segment of the pass is compared with the oracle's brute force
(every beam's group box through the reference's IntersectP, photonbeambvh.h:60-72 +
geometry.h:1410-1436, then photonbeam.cpp:494-508) on sampled segments against the FULL beam set:
contribution counts exactly, per-segment RGB within max(1e-5, 4 u sqrt(n)) of the exact (double)
sum of the oracle's float terms (the reference's own float-order sum is reported beside it, as in
tests/test_c4_gpu.py).  The production film must also equal the per-segment sums added by pixel.
Reference: photonbeam.cpp:354-356, 494-508, 562; src/media/grid.cpp:46-120."""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

R0, ALPHA = 0.01, 0.5


def _full_size_pass(bre, oracle, scene_mod_gpu, tag, width, photons, iteration, nsample, min_contrib):
    import torch

    scene = scene_mod_gpu.cornell_smoke_scene(0.5, 4.5, 0.7, n=64, seed=7)
    R = bre.beam_radius_at(R0, ALPHA, iteration)
    t0 = time.perf_counter()

    def progress(msg):  # a line per phase: a long GPU phase that prints nothing looks hung
        print(f"{tag} [{time.perf_counter() - t0:6.1f} s] {msg}", flush=True)

    with bre.BeamGather(0) as g:
        nb = g.trace_photons(scene, photons, iteration, 5, R)
        n = g.camera_pass(scene, width, width, iteration, 5, True, True)
        progress(f"photon pass {nb} beams, camera pass {n} segments, R {R:.6g}")
        seg_rgb = torch.zeros((n, 3), dtype=torch.float32, device="cuda")
        counts = torch.zeros((n, 2), dtype=torch.int32, device="cuda")
        ld = torch.zeros((width * width, 3), dtype=torch.float32, device="cuda")
        t1 = time.perf_counter()
        g.gather_camera_segments(R, accum=ld, seg_rgb=seg_rgb, counts=counts)
        g.synchronize()
        progress(f"production gather {time.perf_counter() - t1:.2f} s")
        beams = g.get_beams()
        segs = g.get_segments()
    seg_rgb, counts, ld = seg_rgb.cpu().numpy(), counts.cpu().numpy(), ld.cpu().numpy()
    assert (counts[:, 0] == -1).all()
    acc = np.zeros((width * width, 3), np.float64)
    np.add.at(acc, segs["pixel"], seg_rgb.astype(np.float64))
    assert acc.sum() > 0
    assert np.abs(ld - acc).max() <= 1e-5 * max(float(np.abs(acc).max()), 1e-30)
    # the oracle on sampled segments against every beam (16 host threads)
    idx = np.random.default_rng(5000 + iteration).choice(n, nsample, replace=False)
    sample = {k: np.ascontiguousarray(segs[k][idx]) for k in ("o", "p", "d", "tmax")}
    progress(f"oracle brute force: {nsample} segments x {nb} beams")
    ref = oracle.bruteforce(beams, sample, R, nthreads=16)
    progress(f"oracle done, {int(ref['contrib'].sum())} contributions")
    assert ref["contrib"].sum() > min_contrib
    assert np.array_equal(counts[idx, 1], ref["contrib"]), "production contribution counts differ"
    exact = ref["seg_rgb_exact"]
    scale = np.maximum(np.abs(exact).max(axis=1), 1e-30)
    err = np.abs(seg_rgb[idx].astype(np.float64) - exact).max(axis=1) / scale
    tol = np.maximum(1e-5, 4 * 2.0 ** -24 * np.sqrt(ref["contrib"].astype(np.float64)))
    ref_err = np.abs(ref["seg_rgb"].astype(np.float64) - exact).max(axis=1) / scale
    print(f"{tag}: {nb} beams, {n} segments; per-segment error vs the exact sum: GPU max {err.max():.2e}, "
          f"reference-order float sum max {ref_err.max():.2e}; max contributions {int(ref['contrib'].max())}")
    worst = int(np.argmax(err / tol))
    assert (err <= tol).all(), (float(err[worst]), float(tol[worst]), int(ref["contrib"][worst]))
    return nb, n


@pytest.mark.timeout(600)
def test_c3_full_size_iteration0(bre, oracle, scene_mod_gpu):
    nb, n = _full_size_pass(bre, oracle, scene_mod_gpu, "C3", 1024, 5_000_000, 0, 200, 1_000_000)
    assert nb > 10_000_000 and n > 1_000_000


@pytest.mark.timeout(900)
def test_c5_full_photon_count_last_pass(bre, oracle, scene_mod_gpu):
    nb, n = _full_size_pass(bre, oracle, scene_mod_gpu, "C5", 1024, 50_000_000, 9, 100, 100_000)
    assert nb > 100_000_000 and n > 1_000_000
