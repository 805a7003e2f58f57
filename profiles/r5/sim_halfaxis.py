"""CPU model (round 5): the per-lane tile line reject with one axis per tile (today) against one axis
per half tile (32 beams each): a half no lane keeps drops its beams from the scan.  Real C2 packets
(profiles/r5/sim_data.py); bundle = bbox-centre line; axes through the centres of the beams' start /
end boxes, rho from the (unclipped) beam end points; the scan's step count as the kernel picks it.
usage: python profiles/r5/sim_halfaxis.py IT NPACK"""
import sys
import time

import numpy as np

sys.path.insert(0, "profiles/r3b")
from simlib import hilbert_keys, quant, world_bound, ray_box  # noqa: E402

it = int(sys.argv[1]); npk = int(sys.argv[2])
D = np.load(f"/tmp/c2_it{it}.npz")
R = float(D["R"])
bs, be, br = D["bs"].astype(np.float64), D["be"].astype(np.float64), D["br"].astype(np.float64)
so, sp, sd, st = [D[k].astype(np.float64) for k in ("so", "sp", "sd", "st")]
dep = D["sdep"]
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


def axis(ix):
    s, e = bs[ix], be[ix]
    ps = 0.5 * (s.min(0) + s.max(0)); pe = 0.5 * (e.min(0) + e.max(0))
    d = pe - ps; d /= max(np.linalg.norm(d), 1e-30)
    rho = np.linalg.norm(np.cross(np.concatenate([s, e]) - ps, d), axis=1).max()
    return ps, d, rho + maxd[ix].max()


def lanes_near(o, au, ps, d, thr):
    n = np.cross(au, d); nl = np.linalg.norm(n, axis=1)
    t = np.abs(((ps - o) * n).sum(1))
    return ~((nl >= 0.1) & (t / np.maximum(nl, 1e-12) > thr))


def far_bundle(o, p, b0, u, md):
    c_o = 0.5 * (o.min(0) + o.max(0)); c_p = 0.5 * (p.min(0) + p.max(0))
    cu = c_p - c_o; cu /= max(np.linalg.norm(cu), 1e-30)
    X = np.concatenate([o, p])
    delta = np.linalg.norm(np.cross(X - c_o, cu), axis=1).max()
    n = np.cross(cu, u); nl = np.linalg.norm(n, axis=1)
    t = np.abs(((b0 - c_o) * n).sum(1))
    return (nl >= 0.1) & (t / np.maximum(nl, 1e-12) > md + delta)


def cost(on, kept):
    return on if on * 8 < kept * 6 else (kept + 1) // 2


t0 = time.time()
for pi in pk:
    sl = slice(pi * 64, pi * 64 + 64)
    o, p, d, tm = so[sl], sp[sl], sd[sl], st[sl]
    kind = "primary" if (dep[sl] == 0).mean() > 0.5 else "bounce"
    A = p - o; ma = np.linalg.norm(A, axis=1); au = A / np.where(ma > 0, ma, 1)[:, None]
    inv = 1.0 / np.where(d == 0, 1e-30, d)
    hit = ray_box(o, inv, tm, tlo, thi)
    for tt in np.nonzero(hit.any(0))[0]:
        idx = np.arange(tt * 64, min(tt * 64 + 64, nb))
        onl = hit[:, tt]
        add((kind, "visits"), 1)
        keep_b = ~far_bundle(o, p, bs[idx], bu[idx], maxd[idx])
        ps, dd, thr = axis(idx)
        on1 = onl & lanes_near(o, au, ps, dd, thr)
        if on1.any():
            add((kind, "staged1"), 1)
            add((kind, "steps1"), cost(int(on1.sum()), int(keep_b.sum())))
        h = len(idx) // 2
        halves = [idx[:h], idx[h:]] if h > 0 else [idx]
        ons = []
        kept2 = np.zeros(len(idx), bool)
        for hi_, hix in enumerate(halves):
            ps, dd, thr = axis(hix)
            onh = onl & lanes_near(o, au, ps, dd, thr)
            ons.append(onh)
            if onh.any():
                kept2[hi_ * h: hi_ * h + len(hix)] = keep_b[hi_ * h: hi_ * h + len(hix)]
        on2 = np.logical_or.reduce(ons)
        if on2.any():
            add((kind, "staged2"), 1)
            add((kind, "steps2"), cost(int(on2.sum()), int(kept2.sum())))
print("it", it, "R %.5f" % R, "packets", npk, "time %.1f s" % (time.time() - t0))
for kind in ("primary", "bounce"):
    n = tot.get((kind, "visits"), 0)
    if n:
        print(f"{kind}: visits {n}; one axis: staged {tot.get((kind, 'staged1'), 0) / n:.3f} steps/visit "
              f"{tot.get((kind, 'steps1'), 0) / n:.2f};  half axes: staged {tot.get((kind, 'staged2'), 0) / n:.3f} "
              f"steps/visit {tot.get((kind, 'steps2'), 0) / n:.2f}")
