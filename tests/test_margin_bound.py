"""The tile kernel's prefilter margins (bre_gather.hip, scan_keep_mask with margin mode 1) against the
reference's ComputeClosestPoints (photonbeam.cpp:87-186, restated in the oracle).

The kernel rejects a (lane, beam) pair when the separable line-distance test says the two LINES are
more than thr = Ab' + Al' apart.  That is only safe if every distance the reference computes for
such a pair is >= maxd = R + r.  Here the scan values and the test are emulated in float32 (fma by
one rounding of the exact float64 product-sum), pairs are placed just outside the threshold -- with
the closest points inside, before and beyond either segment (the clamp cases and the quirk of
:178-181 that keeps pB on the beam's line) and scenes offset from the origin -- and every rejected
pair's reference distance must be >= maxd.  The pairs just inside the threshold are checked to be
kept, so the test really sits on the boundary."""
import numpy as np
import pytest

from oracle_lib import load_oracle

f32 = np.float32


def fma32(a, b, c):
    return (np.asarray(a, np.float64) * np.asarray(b, np.float64) + np.asarray(c, np.float64)).astype(f32)


def unit_f32(a0, a1):
    """Vector3 A = a1 - a0; magA = Length(A); A / magA (multiply by 1/magA) -- photonbeam.cpp:90-92, 121."""
    A = (a1 - a0).astype(f32)
    mag = np.sqrt(((A[..., 0] * A[..., 0]) + (A[..., 1] * A[..., 1])) + (A[..., 2] * A[..., 2])).astype(f32)
    inv = (f32(1.0) / mag).astype(f32)
    return (A * inv[..., None]).astype(f32), mag


def cross_f32(a, b):  # -ffp-contract=off: products rounded, then the difference
    return np.stack([a[..., 1] * b[..., 2] - a[..., 2] * b[..., 1], a[..., 2] * b[..., 0] - a[..., 0] * b[..., 2],
                     a[..., 0] * b[..., 1] - a[..., 1] * b[..., 0]], -1).astype(f32)


def scan_reject(o, au, mag_a, b0, bu, mag_b, maxd):
    """The reject of scan_keep_mask for margin mode 1 (make_scan_lane / make_scan_beam / staging)."""
    q = cross_f32(o, au)
    o1 = (np.abs(o[..., 0]) + np.abs(o[..., 1]) + np.abs(o[..., 2])).astype(f32)
    al = (f32(1.93e-5) * o1 + f32(1.2e-6) * mag_a).astype(f32)
    m0 = cross_f32(bu, b0)
    b1 = (np.abs(b0[..., 0]) + np.abs(b0[..., 1]) + np.abs(b0[..., 2])).astype(f32)
    ab = (((maxd * f32(1.000001)).astype(f32) + (f32(1.93e-5) * b1).astype(f32)).astype(f32)
          + (f32(2.4e-7) * mag_b).astype(f32)).astype(f32) + f32(1e-6)
    ab = ab.astype(f32)
    c = fma32(au[..., 0], bu[..., 0], fma32(au[..., 1], bu[..., 1], (au[..., 2] * bu[..., 2]).astype(f32)))
    u = fma32(-c, c, f32(1.0001))
    x = fma32(au[..., 0], m0[..., 0], fma32(au[..., 1], m0[..., 1], (au[..., 2] * m0[..., 2]).astype(f32)))
    t = fma32(-bu[..., 0], q[..., 0], fma32(-bu[..., 1], q[..., 1], fma32(-bu[..., 2], q[..., 2], x)))
    # the kernel folds the packet's LARGEST Al' into the beam's staged thr_sq; the lane's own Al' is
    # the least conservative case, so it is the one checked here
    thr = (ab + al).astype(f32)
    thr_sq = (thr * np.abs(thr)).astype(f32)
    lhs = (t * t).astype(f32)
    return (u >= f32(0.0101)) & (lhs > (thr_sq * u).astype(f32)), thr


def ref_distance(ora, a0, a1, b0, b1):
    ok, ac, bc = ora.closest_points(a0, a1, b0, b1)
    if not ok:
        return None
    d = (ac - bc).astype(f32)
    return float(np.sqrt(f32(f32(f32(d[0] * d[0]) + f32(d[1] * d[1])) + f32(d[2] * d[2]))))


@pytest.mark.parametrize("offset,size", [(0.0, 1.0), (0.0, 0.05), (37.0, 2.0), (-300.0, 8.0)])
def test_tight_margins_never_drop_a_reference_contribution(offset, size):
    ora = load_oracle()
    rng = np.random.default_rng(int(abs(offset) * 10 + size * 100))
    n = 6000
    a0 = (offset + size * rng.random((n, 3))).astype(f32)
    a1 = (offset + size * rng.random((n, 3))).astype(f32)
    au, mag_a = unit_f32(a0, a1)
    maxd = (size * 10 ** rng.uniform(-4.5, -1.5, n)).astype(f32)
    # beam direction: random, away from parallel (the test only rejects for |au x bu|^2 >= 1e-2)
    v = rng.normal(size=(n, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    aud = au.astype(np.float64)
    nvec = np.cross(aud, v)
    keep = np.linalg.norm(nvec, axis=1) > 0.11
    nhat = nvec / np.linalg.norm(nvec, axis=1, keepdims=True)
    # closest points of the two lines: on A at t0* (inside, before, beyond), on B at t1* (ditto)
    t0 = mag_a * rng.uniform(-0.3, 1.3, n)
    Lb = size * rng.uniform(0.05, 1.0, n)
    t1 = Lb * rng.uniform(-0.6, 1.6, n)
    # line distance just around the kernel's threshold: estimated margin of mode 1, times 0.5..1.6
    marg = 1.93e-5 * (np.abs(a0).sum(1) * 2 + 0.5 * size) + 1.2e-6 * mag_a + 2.4e-7 * Lb + 1e-6
    D = maxd + marg * rng.uniform(0.5, 1.6, n)
    pa = a0.astype(np.float64) + aud * t0[:, None]
    pb = pa + nhat * D[:, None]
    b0 = (pb - v * t1[:, None]).astype(f32)
    b1 = (pb + v * (Lb - t1)[:, None]).astype(f32)
    bu, mag_b = unit_f32(b0, b1)
    rej, thr = scan_reject(a0, au, mag_a, b0, bu, mag_b, maxd)
    rej &= keep
    checked = 0
    worst = np.inf
    for i in np.nonzero(rej)[0]:
        d = ref_distance(ora, a0[i], a1[i], b0[i], b1[i])
        if d is None:
            continue
        checked += 1
        assert d >= maxd[i], (i, d, maxd[i], thr[i])
        worst = min(worst, (d - maxd[i]) / max(thr[i] - maxd[i], 1e-30))
    # the test sits on the boundary: many pairs are rejected, and many just inside are kept
    assert checked > n // 5
    assert (keep & ~rej).sum() > n // 10
    # the reference distance of every rejected pair clears maxd by a good part of the margin
    print("checked", checked, "kept", int((keep & ~rej).sum()), "worst", worst)
    assert worst > 0.25, worst


def bundle_reject(o, p, au, mag_a, b0, bu, maxd, mag_b):
    """bundle_far_sep (margin mode 1) for one packet: make_bundle's line C and delta in float32,
    then the packet-level line reject of each beam in the separable form."""
    co = (o.astype(np.float64).mean(0)).astype(f32)
    su = au.astype(np.float64).sum(0)
    cu = (su / np.linalg.norm(su)).astype(f32)

    def perp(x):
        t = (x - co).astype(f32)
        c = cross_f32(t, np.broadcast_to(cu, t.shape))
        return np.sqrt(((c * c).sum(-1)).astype(f32)).astype(f32)
    omax = float((np.abs(o).max(1) + mag_a).max())
    cm = float(np.abs(co).max())
    delta = f32(max(perp(o).max(), perp(p).max()) * 1.0001 + 1e-5 * (omax + cm) + 1e-6)
    # bundle_far_sep: the separable form on the staged m0 = bu x b0 and q = co x cu
    cuv = np.broadcast_to(cu, bu.shape)
    m0 = cross_f32(bu, b0)
    q = cross_f32(co[None, :], cu[None, :])[0]
    c = fma32(cuv[:, 0], bu[:, 0], fma32(cuv[:, 1], bu[:, 1], (cuv[:, 2] * bu[:, 2]).astype(f32)))
    u = fma32(-c, c, f32(1.0001))
    x = fma32(cuv[:, 0], m0[:, 0], fma32(cuv[:, 1], m0[:, 1], (cuv[:, 2] * m0[:, 2]).astype(f32)))
    t = fma32(-bu[:, 0], q[0], fma32(-bu[:, 1], q[1], fma32(-bu[:, 2], q[2], x)))
    b1 = np.abs(b0).sum(1).astype(f32)
    col1 = f32(np.abs(co).sum())
    thr = ((maxd + delta) * f32(1.000001) + f32(1.93e-5) * (b1 + col1) + f32(2.5e-6) * f32(omax)
           + f32(2.4e-7) * mag_b + f32(1e-6)).astype(f32)
    return (u >= f32(0.0101)) & ((t * t).astype(f32) > ((thr * thr).astype(f32) * u).astype(f32)), delta, co, cu


@pytest.mark.parametrize("offset,size,spread", [(0.0, 1.0, 0.02), (5.0, 1.0, 0.2), (-80.0, 4.0, 0.05)])
def test_tight_bundle_margins_never_drop_a_reference_contribution(offset, size, spread):
    """Packets of 16 nearly coherent segments (within `spread` of a common line) and beams placed
    just outside the packet-level reject's threshold: no rejected beam may have a lane whose
    reference distance is < maxd, including lanes nearly parallel to the beam."""
    ora = load_oracle()
    rng = np.random.default_rng(int(abs(offset) + 100 * spread))
    checked = rejected = 0
    for _ in range(40):
        c0 = offset + size * rng.random(3)
        dirn = rng.normal(size=3)
        dirn /= np.linalg.norm(dirn)
        L = size * rng.uniform(0.3, 1.0)
        o = (c0 + spread * rng.normal(size=(16, 3))).astype(f32)
        p = (c0 + dirn * L + spread * rng.normal(size=(16, 3))).astype(f32)
        au, mag_a = unit_f32(o, p)
        maxd = f32(size * 10 ** rng.uniform(-4, -1.7))
        nb = 200
        v = rng.normal(size=(nb, 3))
        v[: nb // 4] = dirn + 1e-3 * rng.normal(size=(nb // 4, 3))  # near-parallel to the packet
        v /= np.linalg.norm(v, axis=1, keepdims=True)
        # a first pass fixes C and delta; beams are then placed at D(C, B) around delta + maxd
        _, delta, co, cu = bundle_reject(o, p, au, mag_a, o[:1], au[:1], maxd, mag_a[:1])
        cud = cu.astype(np.float64)
        nvec = np.cross(cud, v)
        ok = np.linalg.norm(nvec, axis=1) > 0.105
        nh = nvec / np.maximum(np.linalg.norm(nvec, axis=1, keepdims=True), 1e-30)
        c1 = float(np.abs(c0).sum()) + 2 * size
        m_est = 2.5e-6 * (np.abs(c0).max() + 2 * size) + 1.93e-5 * 2 * c1 + 1e-6
        D = (float(delta) + float(maxd)) * 1.000001 + m_est * rng.uniform(-1.0, 4.0, nb)
        s0 = rng.uniform(-0.2, 1.2, nb) * L
        pc = co.astype(np.float64) + cud * s0[:, None] + nh * D[:, None]
        Lb = size * rng.uniform(0.05, 1.0, nb)
        t1 = Lb * rng.uniform(-0.6, 1.6, nb)
        b0 = (pc - v * t1[:, None]).astype(f32)
        b1 = (pc + v * (Lb - t1)[:, None]).astype(f32)
        bu, mag_b = unit_f32(b0, b1)
        rej, _, _, _ = bundle_reject(o, p, au, mag_a, b0, bu, np.full(nb, maxd, f32), mag_b)
        rej &= ok
        rejected += int(rej.sum())
        for j in np.nonzero(rej)[0]:
            for i in range(16):
                d = ref_distance(ora, o[i], p[i], b0[j], b1[j])
                if d is None:
                    continue
                checked += 1
                assert d >= maxd, (j, i, d, maxd, delta)
    assert rejected > 500 and checked > 5000
