"""The transcendentals are the reference's own (VERDICT r5 "What's weak" 1).

The reference calls std::exp / std::log / std::sin / std::cos on floats (spectrum.h:222-224 Exp,
homogeneous.cpp:47,59, grid.cpp:76,104, sampling.cpp ConcentricSampleDisk, medium.cpp HG): the host
libm's expf / logf / sinf / cosf.  Until round 6 the GPU and the oracle shared Cephes-style routines
instead (within 2 ulp of libm), so the GPU was bit-exact against the oracle but ~1e-6 away from the
reference-faithful chain.  Since round 6 include/bre_fmath.h returns libm's bits for every float
input (tests/test_fmath_libm.py), so ora_set_libm(1) -- the oracle calling the host libm itself, the
reference's own arithmetic -- changes nothing: the same photons, beams and camera segments bit for
bit, and the GPU image matches that chain to float summation order at a C1-sized and a C3-style
render (over a seeded sample of the film's pixels: the CPU gather of a whole 256^2 film takes tens of
minutes).  With BRE_RECORD=<dir> the GPU tests write their numbers to <dir>/faithful_*.json.
"""
import importlib
import json
import os

import numpy as np
import pytest


@pytest.fixture(scope="module")
def scene_mod():
    return importlib.import_module("beam-radiance-estimate-pbrt_amd.scene")


@pytest.fixture(scope="module")
def torch():
    import torch as t

    return t


def _oracle_chain(oracle, s, w, h, it, photons, depth, R, libm, pixels):
    """The oracle's whole iteration (camera pass, photon pass, SAH tree, gather) with its own
    (include/bre_fmath.h) or the host libm's transcendentals; the gather runs only for the segments of `pixels` (a seeded sample of
    the film -- the full-film CPU gather at these sizes takes tens of minutes), whose radiance
    (surface + media) is returned."""
    oracle.set_libm(libm)
    try:
        cam = oracle.camera_pass(s, w, h, iteration=it, max_depth=depth)
        beams = oracle.trace_photons(s, photons, iteration=it, max_depth=depth, radius=R)
        ld = cam["surface"].astype(np.float64)
        sel = np.isin(cam["pixel"], pixels)
        if sel.any():
            segs = {k: np.ascontiguousarray(cam[k][sel]) for k in ("o", "p", "d", "tmax", "pixel")}
            bvh = oracle.build(beams)
            ld += bvh.gather(segs, R, npix=w * h, nthreads=min(16, os.cpu_count() or 1), chunk=4)["accum"]
            bvh.close()
    finally:
        oracle.set_libm(False)
    return ld[pixels], cam, beams


def _rel_l2(a, b):
    a, b = np.asarray(a, np.float64).ravel(), np.asarray(b, np.float64).ravel()
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def _same_rows(a, b):
    """Fraction of rows (beams / segments) that are bit-identical, when the two sets have one length."""
    if a.shape != b.shape:
        return None
    return float(np.mean(np.all(a.reshape(a.shape[0], -1).view(np.uint32) == b.reshape(b.shape[0], -1).view(np.uint32),
                                axis=1)))


def _record(name, rec):
    d = os.environ.get("BRE_RECORD")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, f"faithful_{name}.json"), "w") as f:
            json.dump(rec, f, indent=1)


def test_libm_switch_changes_nothing(oracle, scene_mod):
    """CPU: the oracle's photon pass with its own transcendentals and with the host libm's: the same
    beams bit for bit (a homogeneous fog and the HG smoke grid, whose delta tracking calls logf on
    every step)."""
    for s in (scene_mod.cornell_scene(), scene_mod.cornell_smoke_scene(n=32)):
        a = oracle.trace_photons(s, 20000, iteration=1, max_depth=5, radius=0.02)
        oracle.set_libm(True)
        try:
            b = oracle.trace_photons(s, 20000, iteration=1, max_depth=5, radius=0.02)
            x = oracle.fmath("exp", np.linspace(-20, 5, 4001, dtype=np.float32))
        finally:
            oracle.set_libm(False)
        y = oracle.fmath("exp", np.linspace(-20, 5, 4001, dtype=np.float32))
        assert np.array_equal(x.view(np.int32), y.view(np.int32))
        assert a["end"].shape[0] > 0 and np.array_equal(a["counts"], b["counts"])
        for k in ("end", "power"):
            assert np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32)), k


CASES = {
    # BASELINE configs[0] / scenes/cornell_fog_c1.pbrt: 256x256, 50k photons, R 0.01, maxdepth 5
    "c1": dict(scene=lambda sm: sm.cornell_scene(), w=256, h=256, photons=50_000, it=0, R0=0.01, npix=1500),
    # BASELINE configs[2] in small: the 64^3 smoke grid, HG g 0.7, 200k photons at 256x256
    "c3": dict(scene=lambda sm: sm.cornell_smoke_scene(n=64), w=256, h=256, photons=200_000, it=0, R0=0.01, npix=600),
}


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(CASES))
def test_gpu_image_against_reference_faithful_oracle(bre, oracle, scene_mod, torch, case):
    c = CASES[case]
    s = c["scene"](scene_mod)
    w, h, photons, it = c["w"], c["h"], c["photons"], c["it"]
    p = scene_mod.render_params(w, h, iterations=1, photons=photons, max_depth=5, radius=c["R0"], alpha=0.5)
    ld = torch.zeros((w * h, 3), dtype=torch.float32, device="cuda")
    with bre.BeamGather(0) as g:
        g.render_iteration(s, p, it, ld)
    torch.cuda.synchronize()
    pixels = np.sort(np.random.default_rng(77).choice(w * h, c["npix"], replace=False))
    got = ld.cpu().numpy().astype(np.float64)[pixels]
    R = np.float32(bre.beam_radius_at(c["R0"], 0.5, it))
    same, cam0, beams0 = _oracle_chain(oracle, s, w, h, it, photons, 5, R, False, pixels)
    ref, cam1, beams1 = _oracle_chain(oracle, s, w, h, it, photons, 5, R, True, pixels)
    rec = {
        "case": case, "width": w, "height": h, "photons": photons, "iteration": it, "R": float(R),
        "pixels_sampled": int(c["npix"]),
        "max_pixel_rel_gpu_vs_libm_oracle": float((np.abs(got - ref).max(1) / np.maximum(np.abs(ref).max(1), 1e-30))[
            np.abs(ref).max(1) > 1e-3 * np.abs(ref).max()].max()),
        "rel_l2_gpu_vs_libm_oracle": _rel_l2(got, ref),
        "rel_l2_gpu_vs_own_fmath_oracle": _rel_l2(got, same),
        "rel_l2_own_fmath_vs_libm_oracle": _rel_l2(same, ref),
        "beams": [int(beams0["end"].shape[0]), int(beams1["end"].shape[0])],
        "segments": [int(cam0["o"].shape[0]), int(cam1["o"].shape[0])],
        "photons_same_beam_count": float(np.mean(beams0["counts"] == beams1["counts"])),
        "beams_bit_identical": _same_rows(beams0["end"], beams1["end"]),
        "segments_bit_identical": _same_rows(cam0["p"], cam1["p"]),
    }
    _record(case, rec)
    print(json.dumps(rec))
    # the libm switch changes no photon and no camera segment: the two oracle chains are one ...
    assert rec["beams_bit_identical"] == 1.0 and rec["segments_bit_identical"] == 1.0, rec
    assert rec["rel_l2_own_fmath_vs_libm_oracle"] == 0.0, rec
    # ... and the GPU is the reference-faithful (libm) chain to float summation order
    assert rec["rel_l2_gpu_vs_libm_oracle"] <= 1e-5, rec
    assert got.mean() > 0
