"""The C++ integrator mirror (host/photonbeam_gpu.h) on the GPU, driven the way
adapters/pbrt/photonbeam.patch drives it: bre_gather_demo builds PhotonBeamGpuBVH from one
iteration's beams (photonbeam.cpp:438), records the camera segments in several SegmentRecorders
(the patch's per-thread recorders, :494-508), calls Gather once per recorder into one pixel Ld
buffer and resolves L = Ld / (iter + 1) (:578).  Input is a real oracle photon pass and camera
pass on the Cornell fog scene; the image must equal the oracle gather's (relative L2 1e-5 plus the
per-pixel bound used for the render tests).  With --devices the mirror runs several libbre contexts
(here all on GPU 0) through bre_set_beams_sharded / bre_gather_sharded -- the one-process multi-GPU
path of the adapter -- and the film must equal the one-context film (1e-6 relative L2: only the
float order of the film sums differs)."""
import importlib
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEMO = os.path.join(ROOT, "beam-radiance-estimate-pbrt_amd", "host", "bre_gather_demo")


def _write(path_b, path_s, beams, segs, npix, R):
    with open(path_b, "wb") as f:
        n = beams["radius"].shape[0]
        np.array([n], np.int64).tofile(f)
        rec = np.concatenate([beams["start"], beams["end"], beams["radius"][:, None], beams["power"]], 1)
        np.ascontiguousarray(rec, np.float32).tofile(f)
    with open(path_s, "wb") as f:
        n = segs["tmax"].shape[0]
        np.array([n, npix], np.int64).tofile(f)
        np.array([R], np.float32).tofile(f)
        dt = np.dtype([("v", "<f4", (10,)), ("pix", "<i4")])
        rec = np.zeros(n, dt)
        rec["v"] = np.concatenate([segs["o"], segs["p"], segs["d"], segs["tmax"][:, None]], 1)
        rec["pix"] = segs["pixel"]
        rec.tofile(f)


def test_demo_lattice_runs():
    assert os.path.exists(DEMO), "build with make -C beam-radiance-estimate-pbrt_amd/host"
    r = subprocess.run([DEMO, "48"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "image sum" in r.stdout


@pytest.mark.parametrize("split,devices", [(1, "0"), (3, "0"), (3, "0,0,0")])
def test_mirror_build_gather_matches_oracle(oracle, tmp_path, split, devices):
    sc = importlib.import_module("beam-radiance-estimate-pbrt_amd.scene")
    s = sc.cornell_scene()
    w, h, it, photons = 48, 40, 2, 20000
    R = np.float32(oracle.radius_at(0.05, 0.5, it))
    cam = oracle.camera_pass(s, w, h, iteration=it, max_depth=5, render_surfaces=False)
    beams = oracle.trace_photons(s, photons, iteration=it, max_depth=5, radius=R)
    segs = {k: cam[k] for k in ("o", "p", "d", "tmax", "pixel")}
    ref = oracle.build(beams).gather(segs, R, npix=w * h)["accum"].astype(np.float64) / (it + 1)
    pb, ps, po = (str(tmp_path / n) for n in ("b.bin", "s.bin", "o.bin"))
    _write(pb, ps, beams, segs, w * h, R)
    r = subprocess.run([DEMO, "--beams", pb, "--segments", ps, "--out", po, "--split", str(split),
                        "--iteration", str(it), "--devices", devices], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    ndev = len(devices.split(","))
    assert f"from {split} recorders in one gather on {ndev} contexts" in r.stdout, r.stdout
    got = np.fromfile(po, np.float32).reshape(-1, 3).astype(np.float64)
    assert got.shape == ref.shape
    assert np.linalg.norm(got - ref) <= 1e-5 * np.linalg.norm(ref)
    mag = np.abs(ref).max(1)
    big = mag > 1e-3 * mag.max()
    assert (np.abs(got - ref).max(1)[big] <= 1e-4 * mag[big]).all()
    assert ref.sum() > 0


def test_mirror_multi_device_equals_one_device(oracle, tmp_path):
    """8 contexts (the 8 GPUs of a node, here all on GPU 0) give the 1-context film."""
    sc = importlib.import_module("beam-radiance-estimate-pbrt_amd.scene")
    s = sc.cornell_scene()
    w, h, it, photons = 64, 64, 0, 30000
    R = np.float32(oracle.radius_at(0.05, 0.5, it))
    cam = oracle.camera_pass(s, w, h, iteration=it, max_depth=5, render_surfaces=False)
    beams = oracle.trace_photons(s, photons, iteration=it, max_depth=5, radius=R)
    segs = {k: cam[k] for k in ("o", "p", "d", "tmax", "pixel")}
    pb, ps = str(tmp_path / "b.bin"), str(tmp_path / "s.bin")
    _write(pb, ps, beams, segs, w * h, R)
    imgs = []
    for devices in ("0", "0,0,0,0,0,0,0,0"):
        po = str(tmp_path / f"o{len(devices)}.bin")
        r = subprocess.run([DEMO, "--beams", pb, "--segments", ps, "--out", po, "--split", "4", "--devices", devices],
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        imgs.append(np.fromfile(po, np.float32).astype(np.float64))
    assert imgs[0].sum() > 0
    assert np.linalg.norm(imgs[1] - imgs[0]) <= 1e-6 * np.linalg.norm(imgs[0])


def test_demo_reports_bad_input(tmp_path):
    p = tmp_path / "bad.bin"
    p.write_bytes(b"\x01")
    r = subprocess.run([DEMO, "--beams", str(p), "--segments", str(p), "--out", str(tmp_path / "o")],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "bad header" in r.stderr
