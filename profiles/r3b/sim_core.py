"""Core/outlier packet bundles (design study): the packet line reject with the bundle of the core
lanes only (the n_out farthest lanes from the packet line left out), the outlier lanes scanned
transposed against every beam the full bundle keeps.  Per sampled C2 packet: scan steps of the
current scheme (kept_all / 2 per visited tile) vs core + outliers (kept_core / 2 + n_out per tile
with any beam kept by the full bundle).  usage: python profiles/r3b/sim_core.py IT NPACK"""
import sys, time, numpy as np
sys.path.insert(0, "profiles/r3b")
from simlib import hilbert_keys, quant, world_bound, ray_box

it = int(sys.argv[1]); npk = int(sys.argv[2])
D = np.load(f"/tmp/c2_it{it}.npz")
R = float(D["R"])
bs, be, br = D["bs"].astype(np.float64), D["be"].astype(np.float64), D["br"].astype(np.float64)
so, sp, sd, st = (D[k].astype(np.float64) for k in ("so", "sp", "sd", "st")); dep = D["sdep"]
pts = np.concatenate([bs, be]); lo, hi = pts.min(0), pts.max(0)
ob = np.argsort(hilbert_keys(np.concatenate([quant(bs, lo, hi), quant(be, lo, hi)], 1)), kind="stable")
bs, be, br = bs[ob], be[ob], br[ob]
blo, bhi = world_bound(bs, be, br)
nb = len(bs); T = (nb + 63) // 64; pad = T * 64 - nb
tlo = np.concatenate([blo, np.full((pad, 3), np.inf)]).reshape(T, 64, 3).min(1)
thi = np.concatenate([bhi, np.full((pad, 3), -np.inf)]).reshape(T, 64, 3).max(1)
bu = (be - bs) / np.linalg.norm(be - bs, axis=1, keepdims=True)
pts = np.concatenate([so, sp]); lo, hi = pts.min(0), pts.max(0)
os_ = np.argsort(hilbert_keys(np.concatenate([quant(so, lo, hi), quant(sp, lo, hi)], 1)), kind="stable")
so, sp, sd, st, dep = so[os_], sp[os_], sd[os_], st[os_], dep[os_]
P = len(so) // 64
rng = np.random.default_rng(1)
maxd = 2 * R
res = {}
t0 = time.time()
for pi in rng.choice(P, npk, replace=False):
    sl = slice(pi * 64, pi * 64 + 64)
    o, p, d, tm = so[sl], sp[sl], sd[sl], st[sl]
    au = (p - o) / np.linalg.norm(p - o, axis=1, keepdims=True)
    inv = 1.0 / np.where(d == 0, 1e-30, d)
    hit = ray_box(o, inv, tm, tlo, thi)
    vis = np.nonzero(hit.any(0))[0]
    idx = (vis[:, None] * 64 + np.arange(64)[None, :]).ravel(); idx = idx[idx < nb]
    tix = np.searchsorted(vis, idx // 64)

    def bundle(sel):
        co = o[sel].mean(0); cu = au[sel].sum(0); cu /= np.linalg.norm(cu)
        perp = lambda x: np.linalg.norm(np.cross(x - co, cu), axis=-1)
        return co, cu, np.maximum(perp(o), perp(p))

    def kept(co, cu, delta):
        n = np.cross(cu, bu[idx]); nn = np.linalg.norm(n, axis=1)
        dist = np.abs(((bs[idx] - co) * n).sum(1)) / np.maximum(nn, 1e-12)
        return (nn < 0.1) | (dist <= delta + maxd)

    co, cu, pl = bundle(np.arange(64))
    k_all = kept(co, cu, pl.max())
    steps_all = np.bincount(tix, weights=k_all, minlength=len(vis))
    res["cur"] = res.get("cur", 0) + np.ceil(steps_all / 2).sum()
    order = np.argsort(pl)
    for nout in (2, 4, 8, 16):
        core = order[:64 - nout]
        co2, cu2, pl2 = bundle(core)
        k_core = kept(co2, cu2, pl2[core].max())
        sc = np.bincount(tix, weights=k_core, minlength=len(vis))
        # outlier lanes: one transposed step per outlier lane on the tile (lane on) with any beam kept
        anyk = steps_all > 0
        onout = hit[np.ix_(order[64 - nout:], vis)].sum(0)
        res[nout] = res.get(nout, 0) + (np.ceil(sc / 2) + np.where(anyk, onout, 0)).sum()
    res["dmax"] = res.get("dmax", 0) + pl.max(); res["d90"] = res.get("d90", 0) + np.percentile(pl, 90)
print("it", it, "packets", npk, "time %.0f s" % (time.time() - t0))
print("mean delta max %.4f  p90 %.4f" % (res["dmax"] / npk, res["d90"] / npk))
for k in (2, 4, 8, 16):
    print("n_out %2d: steps %.3f of the current" % (k, res[k] / res["cur"]))
