"""The .pbrt front end driving the GPU integrator (bre_pbrt_render, bre_render_progressive, the
bre_pbrt command line) on an MI355X.

Bars: the library render of a parsed scene equals bre_render of the same bre_scene put through
Film::SetImage+WriteImage (relative L2 <= 1e-6: only the order of float atomics differs between
runs); against the CPU oracle chain the image is within the north star's 1e-3 relative L2; the
write schedule is the reference's (photonbeam.cpp:564)."""
import ctypes
import importlib
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENES = os.path.join(ROOT, "scenes")


@pytest.fixture(scope="module")
def pb():
    return importlib.import_module("beam-radiance-estimate-pbrt_amd.pbrt")


SMALL = open(os.path.join(SCENES, "cornell_fog_c1.pbrt")).read()
SMALL = (SMALL.replace("[256]", "[48]", 1).replace("[256]", "[40]", 1)
         .replace('"integer iterations" [1]', '"integer iterations" [3]')
         .replace("[50000]", "[20000]").replace('"float initialbeamradius" [0.01]', '"float initialbeamradius" [0.05]')
         .replace('Include "cornell_world.pbrt"', open(os.path.join(SCENES, "cornell_world.pbrt")).read()))


def _rel_l2(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def test_pbrt_render_equals_library_render(bre, pb):
    s = pb.parse_string(SMALL)
    assert s.ok, s.messages
    assert (s.film["xres"], s.film["yres"], s.params.end_iteration) == (48, 40, 3)
    img = s.render(write_files=False)
    with bre.BeamGather(0) as g:
        L = g.render(s.scene, s.params)
    ref = pb.film_finalize(L.reshape(-1, 3)).reshape(L.shape)
    assert img.shape == (40, 48, 3) and img.mean() > 0
    assert _rel_l2(img, ref) <= 1e-6


def test_pbrt_render_matches_oracle(bre, pb, oracle):
    s = pb.parse_string(SMALL)
    w, h, p = s.film["xres"], s.film["yres"], s.params
    img = s.render(write_files=False)
    ld = np.zeros((w * h, 3))
    for it in range(p.end_iteration):
        R = np.float32(bre.beam_radius_at(p.initial_radius, p.alpha, it))
        cam = oracle.camera_pass(s.scene, w, h, iteration=it, max_depth=p.max_depth)
        ld += cam["surface"]
        beams = oracle.trace_photons(s.scene, p.photons_per_iteration, iteration=it, max_depth=p.max_depth, radius=R)
        out = oracle.build(beams).gather({k: cam[k] for k in ("o", "p", "d", "tmax", "pixel")}, R, npix=w * h)
        ld += out["accum"]
    ref = pb.film_finalize((ld / p.end_iteration).astype(np.float32))
    assert _rel_l2(img.reshape(-1, 3), ref) <= 1e-3


def test_progressive_write_schedule(bre):
    sc = importlib.import_module("beam-radiance-estimate-pbrt_amd.scene")
    lib = bre.load_library()
    s = sc.cornell_scene()
    p = sc.render_params(16, 16, iterations=5, photons=4000, max_depth=3, radius=0.05)
    seen = []
    FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_int32, ctypes.POINTER(ctypes.c_float), ctypes.c_void_p)

    def on_image(it, img, user):
        seen.append((it, np.ctypeslib.as_array(img, shape=(16 * 16 * 3,)).copy()))
        return 0

    cb = FN(on_image)
    with bre.BeamGather(0) as g:
        assert lib.bre_render_progressive(g.h, ctypes.addressof(s), ctypes.addressof(p), 2, cb, None) == 0
        final = g.render(s, p)
    # (iter + 1) % 2 == 0 -> iterations 1 and 3; iter + 1 == end -> 4
    assert [it for it, _ in seen] == [1, 3, 4]
    assert _rel_l2(seen[-1][1], final.ravel()) <= 1e-6
    # a callback that refuses stops the render with BRE_ERR_STATE
    stop = FN(lambda it, img, user: 1)
    with bre.BeamGather(0) as g:
        assert lib.bre_render_progressive(g.h, ctypes.addressof(s), ctypes.addressof(p), 1, stop, None) == 4


def test_cli_renders_pfm(pb, tmp_path):
    scene = tmp_path / "small.pbrt"
    scene.write_text(SMALL)
    out = tmp_path / "out.pfm"
    r = subprocess.run([pb.CLI_PATH, "--outfile", str(out), str(scene)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    img = pb.read_pfm(str(out))
    ref = pb.parse_string(SMALL).render(write_files=False)
    assert img.shape == ref.shape and _rel_l2(img, ref) <= 1e-6


def test_big_mesh_pbrt_render_matches_oracle(bre, pb, oracle):
    """12,110 triangles through the .pbrt front end (triangles_ext, the scene BVH on the GPU): the
    render is within the north star's 1e-3 of the oracle chain."""
    from test_pbrt_scene import sphere_pbrt

    k = SMALL.rindex("AttributeBegin")
    s = pb.parse_string(SMALL[:k] + sphere_pbrt() + SMALL[k:])
    assert s.ok, s.messages
    assert s.scene.n_triangles == 12110
    w, h, p = s.film["xres"], s.film["yres"], s.params
    img = s.render(write_files=False)
    ld = np.zeros((w * h, 3))
    for it in range(p.end_iteration):
        R = np.float32(bre.beam_radius_at(p.initial_radius, p.alpha, it))
        cam = oracle.camera_pass(s.scene, w, h, iteration=it, max_depth=p.max_depth)
        ld += cam["surface"]
        beams = oracle.trace_photons(s.scene, p.photons_per_iteration, iteration=it, max_depth=p.max_depth, radius=R)
        out = oracle.build(beams).gather({k: cam[k] for k in ("o", "p", "d", "tmax", "pixel")}, R, npix=w * h)
        ld += out["accum"]
    ref = pb.film_finalize((ld / p.end_iteration).astype(np.float32))
    assert img.mean() > 0
    assert _rel_l2(img.reshape(-1, 3), ref) <= 1e-5


C1 = open(os.path.join(SCENES, "cornell_fog_c1.pbrt")).read().replace(
    'Include "cornell_world.pbrt"', open(os.path.join(SCENES, "cornell_world.pbrt")).read())


def _imgtool_diff(a, b):
    """The reference's `imgtool diff` figures (src/tools/imgtool.cpp:393-432): over the RGB channels
    where either image is nonzero, relative differences |a - b| / a above 0.5% (small) and 5% (big),
    and the relative difference of the two images' means."""
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    nz = ~((a == 0) & (b == 0))
    with np.errstate(divide="ignore", invalid="ignore"):
        d = np.abs(a[nz] - b[nz]) / a[nz]
    avg0, avg1 = a[nz].sum() / a.size, b[nz].sum() / b.size
    return {"small": int(np.sum(d > 0.005)), "big": int(np.sum(d > 0.05)),
            "avg_delta_pct": 100.0 * (avg0 - avg1) / min(avg0, avg1), "channels": int(a.size)}


def _threads():
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return int(omp) if omp.isdigit() and int(omp) > 0 else min(16, len(os.sched_getaffinity(0)))


@pytest.mark.parametrize("arith", ["own", "libm"])
def test_c1_full_image_matches_oracle(bre, pb, oracle, arith):
    """BASELINE configs[0] at its own size: scenes/cornell_fog_c1.pbrt UNMODIFIED (256x256, 50k photons,
    1 iteration, R0 0.01) rendered by bre_pbrt_render on the GPU, against the oracle chain -- camera pass,
    photon pass, the reference's SAH tree and gather (every candidate in DFS order; ora_gather_skip),
    Film::SetImage + WriteImage -- over the whole film.  `own`: the oracle with the transcendentals the
    GPU shares (include/bre_fmath.h); `libm`: with the host libm, the reference's arithmetic -- since
    round 6 the same bits (tests/test_fmath_libm.py).  Either way only float summation order differs:
    within 1e-5 relative L2 (the north star's bar is 1e-3); the imgtool counts are printed beside it."""
    s = pb.parse_string(C1)
    assert s.ok, s.messages
    w, h, p = s.film["xres"], s.film["yres"], s.params
    assert (w, h, p.end_iteration, p.photons_per_iteration, p.max_depth) == (256, 256, 1, 50000, 5)
    assert abs(p.initial_radius - 0.01) < 1e-9
    img = s.render(write_files=False)
    R = np.float32(bre.beam_radius_at(p.initial_radius, p.alpha, 0))
    oracle.set_libm(arith == "libm")
    try:
        cam = oracle.camera_pass(s.scene, w, h, iteration=0, max_depth=p.max_depth)
        beams = oracle.trace_photons(s.scene, p.photons_per_iteration, iteration=0, max_depth=p.max_depth, radius=R)
    finally:
        oracle.set_libm(False)
    out = oracle.build(beams).gather_skip({k: cam[k] for k in ("o", "p", "d", "tmax", "pixel")}, R, npix=w * h,
                                          nthreads=_threads())
    ref = pb.film_finalize((cam["surface"].astype(np.float32) + out["accum"]).astype(np.float32))
    l2 = _rel_l2(img.reshape(-1, 3), ref)
    diff = _imgtool_diff(img.reshape(-1, 3), ref)
    print(f"C1 full film ({arith} oracle): rel-L2 {l2:.3e}, imgtool {diff}, segments {cam['tmax'].shape[0]}, "
          f"beams {beams['radius'].shape[0]}, candidates {int(out['cand'].sum())}, "
          f"contributions {int(out['contrib'].sum())}")
    assert img.mean() > 0
    assert l2 <= 1e-5
