"""CPU model (round 5): how many staged beams the packet-level line reject keeps under other packet
bounds, on real C2 packets (data: profiles/r5/sim_data.py).  Per sampled packet of 64 sorted segments:
the beams of the leaf tiles some lane's ray hits, then
  mean   -- today's bundle line (mean origin, mean direction) and its radius delta
  bbox   -- the line through the centres of the origin / end-point boxes, its own delta
  dir    -- the mean line, with delta replaced by the lanes' spread ALONG the common normal of C and
            the beam (max |(x - co) . n|, x the lanes' end points: a valid bound, see DESIGN)
  frust  -- the mean line with a linear radius r(s) = a + b s along it (lanes' points below it),
            the bound min_s sqrt(D^2 + sin^2 (s - s*)^2) - r(s)
  ideal  -- some lane's segment LINE within maxd (what any line-based packet test keeps at best)
usage: python profiles/r5/sim_bundle.py IT NPACK"""
import sys
import time

import numpy as np

sys.path.insert(0, "profiles/r3b")
from simlib import hilbert_keys, quant, world_bound, ray_box, line_dist  # noqa: E402

it = int(sys.argv[1]); npk = int(sys.argv[2])
D = np.load(f"/tmp/c2_it{it}.npz")
R = float(D["R"])
bs, be, br = D["bs"].astype(np.float64), D["be"].astype(np.float64), D["br"].astype(np.float64)
so, sp, sd, st, dep = (D[k].astype(np.float64) for k in ("so", "sp", "sd", "st")), None, None, None, D["sdep"]
so, sp, sd, st = [D[k].astype(np.float64) for k in ("so", "sp", "sd", "st")]
pts = np.concatenate([bs, be]); lo, hi = pts.min(0), pts.max(0)
ob = np.argsort(hilbert_keys(np.concatenate([quant(bs, lo, hi), quant(be, lo, hi)], 1)), kind="stable")
bs, be, br = bs[ob], be[ob], br[ob]
blo, bhi = world_bound(bs, be, br)
nb = len(bs); T = (nb + 63) // 64; pad = T * 64 - nb
tlo = np.concatenate([blo, np.full((pad, 3), np.inf)]).reshape(T, 64, 3).min(1)
thi = np.concatenate([bhi, np.full((pad, 3), -np.inf)]).reshape(T, 64, 3).max(1)
bvec = be - bs; bmag = np.linalg.norm(bvec, axis=1); bu = bvec / np.where(bmag > 0, bmag, 1)[:, None]
pts = np.concatenate([so, sp]); lo, hi = pts.min(0), pts.max(0)
os_ = np.argsort(hilbert_keys(np.concatenate([quant(so, lo, hi), quant(sp, lo, hi)], 1)), kind="stable")
so, sp, sd, st, dep = so[os_], sp[os_], sd[os_], st[os_], dep[os_]
P = len(so) // 64
pk = np.random.default_rng(1).choice(P, npk, replace=False)
maxd = R + br
tot = {}


def add(k, v):
    tot[k] = tot.get(k, 0) + v


t0 = time.time()
for pi in pk:
    sl = slice(pi * 64, pi * 64 + 64)
    o, p, d, tm = so[sl], sp[sl], sd[sl], st[sl]
    kind = "primary" if (dep[sl] == 0).mean() > 0.5 else "bounce"
    A = p - o; ma = np.linalg.norm(A, axis=1); au = A / np.where(ma > 0, ma, 1)[:, None]
    inv = 1.0 / np.where(d == 0, 1e-30, d)
    hit = ray_box(o, inv, tm, tlo, thi)
    vis = np.nonzero(hit.any(0))[0]
    idx = (vis[:, None] * 64 + np.arange(64)[None, :]).ravel()
    idx = idx[idx < nb]
    b0, u, md = bs[idx], bu[idx], maxd[idx]
    X = np.concatenate([o, p])  # the lanes' end points

    def line_test(co, cu, spread_fn):
        n = np.cross(cu, u); nl = np.linalg.norm(n, axis=1)
        t = np.abs(((b0 - co) * n).sum(1))
        Dcb = t / np.maximum(nl, 1e-12)
        far = (nl >= 0.1) & (Dcb > md + spread_fn(co, cu, n, nl))
        return far, Dcb, nl

    def iso(co, cu, n, nl):
        return np.linalg.norm(np.cross(X - co, cu), axis=1).max()

    def directional(co, cu, n, nl):
        nh = n / np.maximum(nl, 1e-12)[:, None]
        return np.abs((X - co) @ nh.T).max(0)

    co_m = o.mean(0); cu_m = au.sum(0); cu_m /= np.linalg.norm(cu_m)
    far_mean, Dm, nlm = line_test(co_m, cu_m, iso)
    c_o = 0.5 * (o.min(0) + o.max(0)); c_p = 0.5 * (p.min(0) + p.max(0))
    cu_b = c_p - c_o; cu_b /= np.linalg.norm(cu_b)
    far_bbox, _, _ = line_test(c_o, cu_b, iso)
    far_dir, _, _ = line_test(co_m, cu_m, directional)
    # K-direction polygon bound of the directional spread: h_k = max |w . v_k| for K directions v_k in
    # the plane normal to cu (w = x - co), and for a normal n between v_k and v_k+1 (angle theta,
    # spacing phi): |w . n| <= (sin(phi - theta) h_k + sin(theta) h_k+1) / sin(phi)
    e1 = np.cross(cu_m, [1.0, 0.0, 0.0] if abs(cu_m[0]) < 0.9 else [0.0, 1.0, 0.0]); e1 /= np.linalg.norm(e1)
    e2 = np.cross(cu_m, e1)
    W = X - co_m
    wx, wy = W @ e1, W @ e2

    def poly(K):
        ang = np.pi * np.arange(K) / K  # directions over [0, pi): |w.v| is symmetric
        h = np.abs(np.outer(wx, np.cos(ang)) + np.outer(wy, np.sin(ang))).max(0)
        phi = np.pi / K

        def spread(co, cu, n, nl):
            nh = n / np.maximum(nl, 1e-12)[:, None]
            a = np.mod(np.arctan2(nh @ e2, nh @ e1), np.pi)
            k = np.minimum((a / phi).astype(int), K - 1); th = a - k * phi
            return (np.sin(phi - th) * h[k] + np.sin(th) * h[(k + 1) % K]) / np.sin(phi)
        return spread

    far_oct4, _, _ = line_test(co_m, cu_m, poly(4))
    far_oct8, _, _ = line_test(co_m, cu_m, poly(8))
    # today's packet box reject (bundle_box_miss): the rays' capsule around the mean line vs the box
    q = o + d * tm[:, None]
    Xq = np.concatenate([o, q])
    gb = np.linalg.norm(np.cross(Xq - co_m, cu_m), axis=1).max()
    sq = (Xq - co_m) @ cu_m
    c0 = co_m + cu_m * sq.min(); dd = cu_m * (sq.max() - sq.min())
    invc = 1.0 / np.where(dd == 0, 1e-30, dd)
    a_ = (blo[idx] - gb - c0) * invc; b_ = (bhi[idx] + gb - c0) * invc
    miss = np.maximum(np.minimum(a_, b_).max(1), 0) > np.minimum(np.maximum(a_, b_).min(1), 1)
    # frustum along the mean line: s = (x - co) . cu, r = |(x - co) x cu|; upper envelope a + b s
    s_pts = (X - co_m) @ cu_m; r_pts = np.linalg.norm(np.cross(X - co_m, cu_m), axis=1)
    so_, sp_ = s_pts[:64], s_pts[64:]
    ro_, rp_ = r_pts[:64], r_pts[64:]
    bslope = max(0.0, (rp_.max() - ro_.max()) / max(sp_.mean() - so_.mean(), 1e-6))
    a0 = (r_pts - bslope * s_pts).max()
    slo, shi = s_pts.min(), s_pts.max()
    sig = nlm  # |cu x bu|
    # s* on C closest to the beam line: minimise |co + s cu - (b0 + t bu)|
    w0 = co_m - b0; cb = u @ cu_m; dwc = w0 @ cu_m; dwb = (w0 * u).sum(1)
    den = np.maximum(1 - cb * cb, 1e-12)
    sstar = (cb * dwb - dwc) / den

    def g(s):
        return np.sqrt(Dm ** 2 + (sig * (s - sstar)) ** 2) - a0 - bslope * s

    # unconstrained minimiser for b < sig, else the right end; clamp into [slo, shi]
    with np.errstate(invalid="ignore", divide="ignore"):
        u_ = bslope * Dm / (sig * np.sqrt(np.maximum(sig ** 2 - bslope ** 2, 1e-12)))
    smin = np.where(bslope < sig, sstar + u_, shi)
    smin = np.clip(smin, slo, shi)
    fmin = np.minimum(np.minimum(g(smin), g(slo)), g(shi))
    far_fr = (nlm >= 0.1) & (fmin > md)
    # ideal: a lane's line within maxd
    for name, far in (("mean", far_mean), ("bbox", far_bbox), ("dir", far_dir), ("frust", far_fr),
                      ("dir+frust", far_dir | far_fr), ("mean+bbox", far_mean | far_bbox), ("oct4", far_oct4),
                      ("oct8", far_oct8), ("oct4+frust", far_oct4 | far_fr), ("mean|box", far_mean | miss),
                      ("oct8+frust|box", far_oct8 | far_fr | miss), ("dir+frust|box", far_dir | far_fr | miss)):
        add((kind, name), int((~far).sum()))
    add((kind, "staged"), len(idx)); add((kind, "packets"), 1)
print("it", it, "R %.5f" % R, "packets", npk, "time %.1f s" % (time.time() - t0))
for kind in ("primary", "bounce"):
    n = tot.get((kind, "packets"), 0)
    if not n:
        continue
    st_ = tot[(kind, "staged")]
    print(f"{kind}: {n} packets, staged {st_ / n:.0f}/packet; kept fraction of staged:",
          "  ".join(f"{k} {tot[(kind, k)] / st_:.3f}" for k in ("mean", "bbox", "dir", "frust", "dir+frust",
                                                               "mean+bbox", "oct4", "oct8", "oct4+frust",
                                                               "mean|box", "oct8+frust|box", "dir+frust|box")))
