"""CPU model (round 4): the tile kernel's filter funnel over leaf tiles of whole BEAMS (today's tree)
against leaf tiles of beam-LINE CHUNKS (DESIGN.md §12 "Next" item 1), on real C2 data.

    python profiles/r4/sim_chunks.py IT NPACK ELL [ELL ...]      (data: /tmp/c2_itIT.npz, see sim_funnel)

Chunks: every beam's LINE, clipped to the region a contributing pB can lie in (the segments' box grown
by maxd: pB may lie on the line beyond the beam's end, the t1 quirk of photonbeam.cpp:178-181), cut into
pieces of length ELL; a pair belongs to the chunk whose line-parameter interval holds the pair's pB
parameter (the first and last pieces' intervals open to -inf / +inf).  A chunk's box is its piece
grown by maxd, so a lane can contribute through a chunk only if its ray meets that box.  Tiles are 64
consecutive primitives in Hilbert order of (start, end), as the GPU build orders beams.

Per sampled packet of 64 sorted segments, for each index: tiles visited (some lane's ray meets the tile
box), lanes on per visited tile, primitives the packet keeps (line + box rejects, as make_bundle),
(lane, kept primitive) tests, queued pairs (line test), queued pairs per unique contributing pair
(chunk duplicates), and the contributing pairs found (must equal the beam index's).  The per-lane
tile line reject and the transposed scan are not modelled (they apply to both)."""
import sys
import time

import numpy as np

sys.path.insert(0, "profiles/r3b")
from simlib import hilbert_keys, quant, world_bound, ray_box  # noqa: E402


def closest_s(a0, a1, b0, b1):
    """ComputeClosestPoints (photonbeam.cpp:87-186) in float64 -> (ok, dist, sb: pB's parameter on B)."""
    A, Bv = a1 - a0, b1 - b0
    ma, mb = np.linalg.norm(A, axis=-1), np.linalg.norm(Bv, axis=-1)
    au = A / np.where(ma > 0, ma, 1)[..., None]
    bu = Bv / np.where(mb > 0, mb, 1)[..., None]
    cr = np.cross(au, bu)
    den = (cr * cr).sum(-1)
    t = b0 - a0
    det = lambda u, v, w: (u[..., 0] * (v[..., 1] * w[..., 2] - v[..., 2] * w[..., 1])  # noqa: E731
                           - u[..., 1] * (v[..., 0] * w[..., 2] - v[..., 2] * w[..., 0])
                           + u[..., 2] * (v[..., 0] * w[..., 1] - v[..., 1] * w[..., 0]))
    ok = den > 0
    dd = np.where(ok, den, 1)
    t0, t1 = det(t, bu, cr) / dd, det(t, au, cr) / dd
    pA = a0 + au * t0[..., None]
    sb = t1.copy()
    out0 = (t0 < 0) | (t0 > ma)
    pA = np.where((t0 < 0)[..., None], a0, np.where((t0 > ma)[..., None], a1, pA))
    dp = np.clip((bu * (pA - b0)).sum(-1), 0, mb)
    sb = np.where(out0, dp, sb)
    pB = b0 + bu * sb[..., None]
    out1 = (t1 < 0) | (t1 > mb)
    da = np.clip((au * (pB - a0)).sum(-1), 0, ma)
    pA = np.where(out1[..., None], a0 + au * da[..., None], pA)
    return ok, np.linalg.norm(pA - pB, axis=-1), sb


def line_dist(ao, au, bo, bu):
    n = np.cross(au, bu)
    nn = np.linalg.norm(n, axis=-1)
    tn = np.abs(((bo - ao) * n).sum(-1))
    return np.where(nn > 0.1, tn / np.where(nn > 0, nn, 1), 0.0)


def tiles_of(ps, pe, lo, hi):
    """Hilbert (start, end) order, tiles of 64: (order, tile lo, tile hi)."""
    pts = np.concatenate([ps, pe])
    qlo, qhi = pts.min(0), pts.max(0)
    k = hilbert_keys(np.concatenate([quant(ps, qlo, qhi), quant(pe, qlo, qhi)], 1))
    order = np.argsort(k, kind="stable")
    n = len(order)
    T = (n + 63) // 64
    pad = T * 64 - n
    tlo = np.concatenate([lo[order], np.full((pad, 3), np.inf)]).reshape(T, 64, 3).min(1)
    thi = np.concatenate([hi[order], np.full((pad, 3), -np.inf)]).reshape(T, 64, 3).max(1)
    return order, tlo, thi


def main():
    it, npk = int(sys.argv[1]), int(sys.argv[2])
    ells = [float(x) for x in sys.argv[3:]] or [0.25]
    D = np.load(f"/tmp/c2_it{it}.npz")
    R = float(D["R"])
    bs, be, br = D["bs"].astype(np.float64), D["be"].astype(np.float64), D["br"].astype(np.float64)
    so, sp, sd, st = (D[k].astype(np.float64) for k in ("so", "sp", "sd", "st"))
    maxd = R + br
    mmax = float(maxd.max())
    blen = np.linalg.norm(be - bs, axis=1)
    ok_b = blen > 0
    bs, be, br, maxd, blen = bs[ok_b], be[ok_b], br[ok_b], maxd[ok_b], blen[ok_b]
    bu = (be - bs) / blen[:, None]
    blo, bhi = world_bound(bs, be, br)  # the reference's beam box (exact-stage box test)
    # segments: Hilbert (o, p) order, packets of 64, a sample of them
    pts = np.concatenate([so, sp])
    ks = hilbert_keys(np.concatenate([quant(so, pts.min(0), pts.max(0)), quant(sp, pts.min(0), pts.max(0))], 1))
    os_ = np.argsort(ks, kind="stable")
    so, sp, sd, st = so[os_], sp[os_], sd[os_], st[os_]
    P = len(so) // 64
    pk = np.random.default_rng(1).choice(P, npk, replace=False)
    rlo = np.minimum(so.min(0), sp.min(0)) - mmax * 1.01 - 1e-6
    rhi = np.maximum(so.max(0), sp.max(0)) + mmax * 1.01 + 1e-6

    # index A: whole beams
    oA, tloA, thiA = tiles_of(bs, be, blo, bhi)
    idxA = dict(kind="beams", beam=oA, ps=bs[oA], pe=be[oA], lo=blo[oA], hi=bhi[oA], slo=None, shi=None,
                tlo=tloA, thi=thiA)
    indexes = [idxA]
    # index B: line chunks of length ell
    inv = 1.0 / np.where(bu == 0, 1e-300, bu)
    a = (rlo - bs) * inv
    b = (rhi - bs) * inv
    ta, tb = np.minimum(a, b).max(1), np.maximum(a, b).min(1)
    for ell in ells:
        t0 = time.time()
        live = tb > ta
        nch = np.where(live, np.ceil((tb - ta) / ell).astype(np.int64), 0)
        beam = np.repeat(np.arange(len(bs)), nch)
        first = np.repeat(np.cumsum(nch) - nch, nch)
        k = np.arange(len(beam)) - first
        s0 = ta[beam] + k * ell
        s1 = np.minimum(s0 + ell, tb[beam])
        ps = bs[beam] + bu[beam] * s0[:, None]
        pe = bs[beam] + bu[beam] * s1[:, None]
        g = maxd[beam][:, None] * 1.001 + 1e-6
        lo, hi = np.minimum(ps, pe) - g, np.maximum(ps, pe) + g
        slo = np.where(k == 0, -np.inf, s0)
        shi = np.where(k == nch[beam] - 1, np.inf, s1)
        order, tlo, thi = tiles_of(ps, pe, lo, hi)
        indexes.append(dict(kind=f"chunks ell={ell}", beam=beam[order], ps=ps[order], pe=pe[order], lo=lo[order],
                            hi=hi[order], slo=slo[order], shi=shi[order], tlo=tlo, thi=thi))
        print(f"chunks ell={ell}: {len(beam)} ({len(beam) / len(bs):.2f} per beam), built in {time.time() - t0:.0f} s",
              flush=True)
    tot = [dict() for _ in indexes]
    ref_contrib = {}
    t0 = time.time()
    for pi in pk:
        sl = slice(pi * 64, pi * 64 + 64)
        o, p, d, tm = so[sl], sp[sl], sd[sl], st[sl]
        A = p - o
        ma = np.linalg.norm(A, axis=1)
        au = A / np.where(ma > 0, ma, 1)[:, None]
        invd = 1.0 / np.where(d == 0, 1e-30, d)
        # packet bundle (make_bundle)
        co = o.mean(0)
        su = au.sum(0)
        cu = su / np.linalg.norm(su)
        perp = lambda x: np.linalg.norm(np.cross(x - co, cu), axis=-1)  # noqa: E731
        delta = max(perp(o).max(), perp(p).max()) + 1e-6
        q = o + d * tm[:, None]
        gb = max(perp(o).max(), perp(q).max()) + 1e-6
        so_ = ((o - co) * cu).sum(1)
        sq = ((q - co) * cu).sum(1)
        s0, s1 = min(so_.min(), sq.min()) - 1e-6, max(so_.max(), sq.max()) + 1e-6
        for ii, X in enumerate(indexes):
            tt = tot[ii]
            hit = ray_box(o, invd, tm, X["tlo"], X["thi"])  # (64, T)
            vis = np.nonzero(hit.any(0))[0]
            tt["tiles"] = tt.get("tiles", 0) + len(vis)
            tt["on_lanes"] = tt.get("on_lanes", 0) + int(hit[:, vis].sum())
            idx = (vis[:, None] * 64 + np.arange(64)[None, :]).ravel()
            idx = idx[idx < len(X["beam"])]
            bj = X["beam"][idx]
            # packet line reject on the beam's line, box reject on the primitive's box
            n = np.cross(cu, bu[bj])
            nn = (n * n).sum(1)
            tn = np.abs(((bs[bj] - co) * n).sum(1))
            far = (nn >= 1e-2) & (tn > (maxd[bj] + delta) * np.sqrt(nn) + 1e-6)
            c0 = co + cu * s0
            dd = cu * (s1 - s0)
            ic = 1.0 / np.where(dd == 0, 1e-30, dd)
            aa = (X["lo"][idx] - gb - c0) * ic
            bb = (X["hi"][idx] + gb - c0) * ic
            miss = np.maximum(np.minimum(aa, bb).max(1), 0) > np.minimum(np.maximum(aa, bb).min(1), 1)
            keep = ~(far | miss)
            kidx, kb = idx[keep], bj[keep]
            on = hit[:, kidx // 64]  # (64, K): lanes on the kept primitive's tile
            tt["staged"] = tt.get("staged", 0) + len(idx)
            tt["kept"] = tt.get("kept", 0) + len(kidx)
            tt["lane_tests"] = tt.get("lane_tests", 0) + int(on.sum())
            L, K = np.nonzero(on)
            b = kb[K]
            ld = line_dist(o[L], au[L], bs[b], bu[b])
            qd = ld <= maxd[b] * 1.0001 + 1e-5
            L, K, b = L[qd], K[qd], b[qd]
            tt["queued"] = tt.get("queued", 0) + len(L)
            # exact: the reference's box test on the BEAM box, closest points, distance
            a_ = (blo[b] - o[L]) * invd[L]
            b_ = (bhi[b] - o[L]) * invd[L]
            tn_ = np.minimum(a_, b_).max(1)
            tf_ = np.maximum(a_, b_).min(1) * (1 + 6 * 2**-24)
            boxhit = (tn_ <= tf_) & (tn_ < tm[L]) & (tf_ > 0)
            okc, dist, sb = closest_s(o[L], p[L], bs[b], be[b])
            con = boxhit & okc & (dist < maxd[b])
            if X["slo"] is not None:
                pidx = kidx[K]
                own = (sb >= X["slo"][pidx]) & (sb < X["shi"][pidx])
                tt["contrib_dup"] = tt.get("contrib_dup", 0) + int(con.sum())
                con = con & own
            pairs = set(zip((pi * 64 + L[con]).tolist(), b[con].tolist()))
            tt["contrib"] = tt.get("contrib", 0) + len(pairs)
            if ii == 0:
                ref_contrib[pi] = pairs
            else:
                tt["missed"] = tt.get("missed", 0) + len(ref_contrib[pi] - pairs)
                tt["extra"] = tt.get("extra", 0) + len(pairs - ref_contrib[pi])
    print(f"it {it} R {R:.5f} packets {npk} ({time.time() - t0:.0f} s)")
    for X, tt in zip(indexes, tot):
        q = max(tt["queued"], 1)
        print(f"{X['kind']:>18}: prims {len(X['beam'])}  per packet: tiles {tt['tiles'] / npk:.0f}, lanes on/tile "
              f"{tt['on_lanes'] / max(tt['tiles'], 1):.1f}, staged {tt['staged'] / npk:.0f}, kept {tt['kept'] / npk:.0f}, "
              f"lane tests {tt['lane_tests'] / npk:.0f}, queued {tt['queued'] / npk:.0f}, contrib {tt['contrib'] / npk:.0f}; "
              f"tests/queued {tt['lane_tests'] / q:.1f}, contrib/queued {tt['contrib'] / q:.3f}"
              + (f", dup-contrib/contrib {tt['contrib_dup'] / max(tt['contrib'], 1):.2f}, missed {tt['missed']}, extra {tt['extra']}"
                 if X["slo"] is not None else ""))


if __name__ == "__main__":
    main()
