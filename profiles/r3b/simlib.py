"""CPU model of the tile kernel's filter funnel on real C2 data (beams and camera segments from the
oracle's photon and camera passes).  Used to size structural changes before they go to the GPU:
per sampled packet of 64 sorted segments it counts visited leaf tiles, staged beams, packet-kept
beams, (lane, kept beam) prefilter tests, queued pairs and contributions, like the GPU counters."""
import numpy as np


def hilbert_keys(q, B=10):
    """Skilling's transpose Hilbert index (bre_math.h hilbert_key<N, B>) of uint coords q (n, N)."""
    x = q.astype(np.uint64).copy()
    n, N = x.shape
    M = np.uint64(1 << (B - 1))
    Q = M
    while Q > 1:
        P = np.uint64(Q - 1)
        for i in range(N):
            has = (x[:, i] & Q) != 0
            x0 = x[:, 0].copy()
            # invert where has
            x[:, 0] = np.where(has, x0 ^ P, x0)
            # exchange where not has
            t = (x0 ^ x[:, i]) & P
            if i == 0:
                pass  # exchange with itself: no-op
            else:
                nh = ~has
                x[:, 0] = np.where(nh, x0 ^ t, x[:, 0])
                x[:, i] = np.where(nh, x[:, i] ^ t, x[:, i])
        Q = np.uint64(Q >> np.uint64(1))
    for i in range(1, N):
        x[:, i] ^= x[:, i - 1]
    t = np.zeros(n, np.uint64)
    Q = M
    while Q > 1:
        t = np.where((x[:, N - 1] & Q) != 0, t ^ np.uint64(Q - 1), t)
        Q = np.uint64(Q >> np.uint64(1))
    for i in range(N):
        x[:, i] ^= t
    key = np.zeros(n, np.uint64)
    for bit in range(B - 1, -1, -1):
        for i in range(N):
            key = (key << np.uint64(1)) | ((x[:, i] >> np.uint64(bit)) & np.uint64(1))
    return key


def quant(x, lo, hi, bits=10):
    ext = np.where(hi - lo > 0, hi - lo, 1.0)
    m = (1 << bits) - 1
    return np.clip(((x - lo) / ext * m + 0.5).astype(np.int64), 0, m)


def world_bound(s, e, r):
    d = e - s
    c = s + d / 2
    ln = np.linalg.norm(d, axis=1, keepdims=True)
    du = d / np.where(ln > 0, ln, 1)
    size = du * ln + 2 * r[:, None] * np.sqrt(np.maximum(1 - du * du, 0))
    p1, p2 = c - size / 2, c + size / 2
    return np.minimum(p1, p2), np.maximum(p1, p2)


def ray_box(o, inv, tmax, lo, hi):
    """o, inv, tmax: (L, 3), (L, 3), (L,); lo, hi: (T, 3) -> hit (L, T)."""
    a = (lo[None, :, :] - o[:, None, :]) * inv[:, None, :]
    b = (hi[None, :, :] - o[:, None, :]) * inv[:, None, :]
    tn = np.minimum(a, b).max(2)
    tf = np.maximum(a, b).min(2) * (1 + 2 * 3 * 2**-24)
    return (tn <= tf) & (tn < tmax[:, None]) & (tf > 0)


def closest_dist(a0, a1, b0, b1):
    """ComputeClosestPoints (photonbeam.cpp:87-186) in float64, vectorised; -> (ok, dist)."""
    A = a1 - a0
    Bv = b1 - b0
    ma = np.linalg.norm(A, axis=-1)
    mb = np.linalg.norm(Bv, axis=-1)
    au = A / np.where(ma > 0, ma, 1)[..., None]
    bu = Bv / np.where(mb > 0, mb, 1)[..., None]
    cr = np.cross(au, bu)
    den = (cr * cr).sum(-1)
    t = b0 - a0
    detA = np.linalg.det(np.stack([t, bu, cr], -2)) if False else (
        t[..., 0] * (bu[..., 1] * cr[..., 2] - bu[..., 2] * cr[..., 1])
        - t[..., 1] * (bu[..., 0] * cr[..., 2] - bu[..., 2] * cr[..., 0])
        + t[..., 2] * (bu[..., 0] * cr[..., 1] - bu[..., 1] * cr[..., 0]))
    detB = (t[..., 0] * (au[..., 1] * cr[..., 2] - au[..., 2] * cr[..., 1])
            - t[..., 1] * (au[..., 0] * cr[..., 2] - au[..., 2] * cr[..., 0])
            + t[..., 2] * (au[..., 0] * cr[..., 1] - au[..., 1] * cr[..., 0]))
    ok = den > 0
    dd = np.where(ok, den, 1)
    t0, t1 = detA / dd, detB / dd
    pA = a0 + au * t0[..., None]
    pB = b0 + bu * t1[..., None]
    pA = np.where((t0 < 0)[..., None], a0, np.where((t0 > ma)[..., None], a1, pA))
    out0 = (t0 < 0) | (t0 > ma)
    dp = np.clip((bu * (pA - b0)).sum(-1), 0, mb)
    pB = np.where(out0[..., None], b0 + bu * dp[..., None], pB)
    out1 = (t1 < 0) | (t1 > mb)
    da = np.clip((au * (pB - a0)).sum(-1), 0, ma)
    pA = np.where(out1[..., None], a0 + au * da[..., None], pA)
    return ok, np.linalg.norm(pA - pB, axis=-1)


def line_dist(ao, au, bo, bu):
    """Distance between infinite lines (broadcasting); near-parallel -> 0 (never rejected)."""
    n = np.cross(au, bu)
    nn = np.linalg.norm(n, axis=-1)
    tn = np.abs(((bo - ao) * n).sum(-1))
    return np.where(nn > 0.1, tn / np.where(nn > 0, nn, 1), 0.0)
