"""The GPU's expf / logf / sinf / cosf (include/bre_fmath.h compiled for gfx950; bre_device_check kind
9 runs the very device functions the photon and camera passes call) against the host's: the same
bits as the oracle's host build of bre_fmath.h, which equals the host glibc libm for every float input
(tests/test_fmath_libm.py), and as the libm itself on a sample.  Inputs: a sweep of every 4099th float
bit pattern (every exponent, both signs, subnormals, infinities and NaNs) and dense samples of the
ranges the passes use (log(1 - u), exp(-sigma_t t), angles in [-pi, 2 pi])."""
import ctypes
import ctypes.util

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KINDS = ("exp", "log", "sin", "cos")


def _inputs():
    sweep = np.arange(0, 1 << 32, 4099, dtype=np.uint64).astype(np.uint32).view(np.float32)
    rng = np.random.default_rng(9)
    dense = np.concatenate([
        rng.random(200_000, dtype=np.float32),                       # 1 - u, u
        -rng.uniform(0, 104, 200_000).astype(np.float32),            # exp(-sigma_t t), down to underflow
        rng.uniform(-np.pi, 2 * np.pi, 200_000).astype(np.float32),  # HG phi, disk angles
        np.array([0.0, -0.0, 1.0, 88.0, 88.72283, 88.7229, -103.97, -104.0, 120.0, -120.0, 1e-30, 1e-45],
                 np.float32),
    ])
    return np.concatenate([sweep, dense]).astype(np.float32)


def _same(a, b):
    ua, ub = a.view(np.uint32), b.view(np.uint32)
    return (ua == ub) | (np.isnan(a) & np.isnan(b))


def test_device_fmath_equals_host(bre, oracle):
    x = _inputs()
    with bre.BeamGather(0) as g:
        y = g.device_check(9, x)
    assert y.shape == (x.shape[0], 4)
    for k, name in enumerate(KINDS):
        ref = oracle.fmath(name, x)
        ok = _same(y[:, k], ref)
        bad = np.flatnonzero(~ok)
        assert bad.size == 0, (name, bad.size, [(float(x[i]), float(y[i, k]), float(ref[i])) for i in bad[:5]])


def test_device_fmath_equals_host_libm_sample(bre):
    libm = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
    fns = []
    for name in ("expf", "logf", "sinf", "cosf"):
        f = getattr(libm, name)
        f.argtypes = [ctypes.c_float]
        f.restype = ctypes.c_float
        fns.append(f)
    x = _inputs()[:: 97].copy()
    with bre.BeamGather(0) as g:
        y = g.device_check(9, x)
    for k, f in enumerate(fns):
        ref = np.array([f(float(v)) for v in x], np.float32)
        assert _same(y[:, k], ref).all(), KINDS[k]
