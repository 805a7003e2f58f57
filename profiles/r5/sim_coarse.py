"""CPU model (round 5, VERDICT r4 item 1's coarse reject): a per-(lane, beam) test in front of the scan's
fp32 test saves a scan step only when it rejects the beam for EVERY on lane of the wave (a wave64
instruction stream runs while any lane needs it).  On real C2 packets (profiles/r5/sim_data.py) this
counts, per kept beam of a visited tile (bbox bundle): the on lanes whose segment LINE is within
maxd * (1 + slack) of the beam line (what a coarse test with that relative slack keeps), and how many
kept beams keep at least one such lane (= fp32 steps the coarse test cannot skip).
usage: python profiles/r5/sim_coarse.py IT NPACK"""
import sys
import time

import numpy as np

sys.path.insert(0, "profiles/r3b")
sys.path.insert(0, "profiles/r5")
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
SL = (0.0, 0.25, 1.0)
tot = {}


def add(k, v):
    tot[k] = tot.get(k, 0) + v


def far_bundle(o, p, b0, u, md):
    c_o = 0.5 * (o.min(0) + o.max(0)); c_p = 0.5 * (p.min(0) + p.max(0))
    cu = c_p - c_o; cu /= max(np.linalg.norm(cu), 1e-30)
    X = np.concatenate([o, p])
    delta = np.linalg.norm(np.cross(X - c_o, cu), axis=1).max()
    n = np.cross(cu, u); nl = np.linalg.norm(n, axis=1)
    t = np.abs(((b0 - c_o) * n).sum(1))
    return (nl >= 0.1) & (t / np.maximum(nl, 1e-12) > md + delta)


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
        kb = ~far_bundle(o, p, bs[idx], bu[idx], maxd[idx])
        if not kb.any():
            continue
        ix = idx[kb]
        n = np.cross(au[:, None, :], bu[ix][None, :, :]); nl = np.linalg.norm(n, axis=2)
        tn = np.abs(((bs[ix][None] - o[:, None]) * n).sum(2))
        dl = tn / np.maximum(nl, 1e-12)
        add((kind, "kept"), len(ix))
        add((kind, "lanetests"), int(onl.sum()) * len(ix))
        for s_ in SL:
            near = ((nl < 0.1) | (dl <= maxd[ix][None] * (1 + s_))) & onl[:, None]
            add((kind, f"pass{s_}"), int(near.sum()))
            add((kind, f"beams{s_}"), int(near.any(0).sum()))
print("it", it, "R %.5f" % R, "packets", npk, "time %.1f s" % (time.time() - t0))
for kind in ("primary", "bounce"):
    k = tot.get((kind, "kept"), 0)
    if k:
        print(f"{kind}: kept beams {k}, lane tests {tot[(kind, 'lanetests')]}; " + "  ".join(
            f"slack {s_:g}: pairs kept {tot[(kind, f'pass{s_}')] / tot[(kind, 'lanetests')]:.4f}, "
            f"beams with a kept lane {tot[(kind, f'beams{s_}')] / k:.3f}" for s_ in SL))
