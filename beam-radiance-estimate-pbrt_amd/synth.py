"""Synthetic workloads for the beam gather (SURVEY.md §8d "synthetic-fog").

Random numbers come from pbrt's PCG32 (src/core/rng.h:60-144), one stream per element:
element i of a workload seeded with `seed` uses ``RNG.SetSequence((seed << 32) | i)``, so any
subset of a workload can be regenerated independently (and by every rank of a multi-GPU run
without communication).  The generator is vectorised over streams with numpy uint64 arithmetic.

Workloads
---------
* ``fog_beams(n, seed=12345, radius=0.01)`` — beams with start ~ U[0,1)^3, direction uniform on
  S^2, length ~ Exp(mean 0.25) clipped to the unit cube (and to >= 1e-3 so no beam is
  degenerate), powerEnd ~ U[0,1)^3.
* ``camera_segments(w, h, seed=777)`` — one segment per pixel: ray from (0.5, 0.5, -1) through a
  jittered point of pixel (x, y) on the z=0 plane, ending where it reaches z = 1
  (``tMax = 2 / d.z``, ``p = o + tMax * d``), d normalised; pixel index ``y * w + x``.
* ``bounce_segments(n, seed=778)`` — incoherent segments: origin U[0,1)^3, direction uniform on
  S^2, ending at the cube boundary (like camera paths after a diffuse bounce).
"""
from __future__ import annotations

import numpy as np

PCG32_DEFAULT_STATE = np.uint64(0x853C49E6748FEA9B)
PCG32_MULT = np.uint64(0x5851F42D4C957F2D)
ONE_MINUS_EPSILON = np.float32(np.nextafter(np.float32(1.0), np.float32(0.0)))


class PCG32:
    """pbrt's RNG (rng.h) vectorised over independent sequences."""

    def __init__(self, seqs: np.ndarray):
        seqs = np.asarray(seqs, dtype=np.uint64)
        self.inc = (seqs << np.uint64(1)) | np.uint64(1)
        self.state = np.zeros_like(seqs)
        with np.errstate(over="ignore"):
            self.uint32()
            self.state = self.state + PCG32_DEFAULT_STATE
            self.uint32()

    def uint32(self) -> np.ndarray:
        old = self.state
        with np.errstate(over="ignore"):
            self.state = old * PCG32_MULT + self.inc
        xorshifted = (((old >> np.uint64(18)) ^ old) >> np.uint64(27)).astype(np.uint32)
        rot = (old >> np.uint64(59)).astype(np.uint32)
        return (xorshifted >> rot) | (xorshifted << ((np.uint32(0) - rot) & np.uint32(31)))

    def uniform(self) -> np.ndarray:
        # std::min(OneMinusEpsilon, Float(UniformUInt32() * 0x1p-32f))
        u = self.uint32().astype(np.float32) * np.float32(2.0**-32)
        return np.minimum(u, ONE_MINUS_EPSILON)


def _streams(seed: int, n: int, offset: int = 0) -> PCG32:
    idx = np.arange(offset, offset + n, dtype=np.uint64)
    return PCG32((np.uint64(seed) << np.uint64(32)) | idx)


def _unit_sphere(u1: np.ndarray, u2: np.ndarray) -> np.ndarray:
    z = 1.0 - 2.0 * u1.astype(np.float64)
    r = np.sqrt(np.maximum(0.0, 1.0 - z * z))
    phi = 2.0 * np.pi * u2.astype(np.float64)
    return np.stack([r * np.cos(phi), r * np.sin(phi), z], axis=1)


def _exit_distance(o: np.ndarray, d: np.ndarray) -> np.ndarray:
    """Distance from o (inside [0,1]^3) along unit d to the cube boundary."""
    with np.errstate(divide="ignore", invalid="ignore"):
        t_hi = np.where(d > 0, (1.0 - o) / d, np.inf)
        t_lo = np.where(d < 0, (0.0 - o) / d, np.inf)
    return np.minimum(t_hi, t_lo).min(axis=1)


def fog_beams(n: int, seed: int = 12345, radius: float = 0.01, mean_length: float = 0.25, offset: int = 0):
    """Return dict of float32 arrays start (n,3), end (n,3), radius (n,), power (n,3)."""
    rng = _streams(seed, n, offset)
    start = np.stack([rng.uniform(), rng.uniform(), rng.uniform()], axis=1).astype(np.float64)
    d = _unit_sphere(rng.uniform(), rng.uniform())
    length = -mean_length * np.log1p(-rng.uniform().astype(np.float64))
    length = np.minimum(length, _exit_distance(start, d))
    length = np.maximum(length, 1e-3)
    end = start + d * length[:, None]
    power = np.stack([rng.uniform(), rng.uniform(), rng.uniform()], axis=1)
    return {
        "start": np.ascontiguousarray(start, dtype=np.float32),
        "end": np.ascontiguousarray(end, dtype=np.float32),
        "radius": np.full(n, radius, dtype=np.float32),
        "power": np.ascontiguousarray(power, dtype=np.float32),
    }


def camera_segments(w: int, h: int, seed: int = 777, pixels: np.ndarray | None = None):
    """One camera segment per pixel (or per listed pixel index)."""
    if pixels is None:
        pixels = np.arange(w * h, dtype=np.int64)
    pixels = np.asarray(pixels, dtype=np.int64)
    n = pixels.shape[0]
    rng = PCG32((np.uint64(seed) << np.uint64(32)) | pixels.astype(np.uint64))
    jx, jy = rng.uniform(), rng.uniform()
    x = (pixels % w).astype(np.float64)
    y = (pixels // w).astype(np.float64)
    q = np.stack([(x + jx) / w, (y + jy) / h, np.zeros(n)], axis=1)
    o = np.tile(np.array([0.5, 0.5, -1.0]), (n, 1))
    d = q - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o32 = o.astype(np.float32)
    d32 = d.astype(np.float32)
    tmax = (np.float32(2.0) / d32[:, 2]).astype(np.float32)
    p32 = (o32 + d32 * tmax[:, None]).astype(np.float32)
    return {
        "o": np.ascontiguousarray(o32),
        "p": np.ascontiguousarray(p32),
        "d": np.ascontiguousarray(d32),
        "tmax": np.ascontiguousarray(tmax),
        "pixel": pixels.astype(np.int32),
    }


def bounce_segments(n: int, seed: int = 778, npix: int | None = None):
    """Incoherent segments inside the unit cube, pixel = i mod npix."""
    rng = _streams(seed, n)
    o = np.stack([rng.uniform(), rng.uniform(), rng.uniform()], axis=1).astype(np.float64)
    d = _unit_sphere(rng.uniform(), rng.uniform())
    t = _exit_distance(o, d)
    o32 = o.astype(np.float32)
    d32 = d.astype(np.float32)
    t32 = t.astype(np.float32)
    p32 = (o32 + d32 * t32[:, None]).astype(np.float32)
    npix = n if npix is None else npix
    return {
        "o": np.ascontiguousarray(o32),
        "p": np.ascontiguousarray(p32),
        "d": np.ascontiguousarray(d32),
        "tmax": np.ascontiguousarray(t32),
        "pixel": (np.arange(n) % npix).astype(np.int32),
    }


def tile_pixels(w: int, h: int, rank: int, world: int, tile: int = 16) -> np.ndarray:
    """Pixels of the 16x16 tiles owned by `rank` (see dist.tile_pixels)."""
    from .dist import tile_pixels as _tp

    return _tp(w, h, rank, world, tile)
