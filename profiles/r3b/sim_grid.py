"""CPU model of a uniform-grid beam index (design study): beams inserted into the cells their
capsule (line piece, radius maxd) can reach, by major-axis slabs; camera segments cut into per-cell
pieces; per cell, every piece tested against every inserted beam.  Reports lane slots (64-piece
packets x list length), line-prefilter survivors and owned contributions for sampled cells.
usage: python profiles/r3b/sim_grid.py IT H NCELLS"""
import sys, time, numpy as np
sys.path.insert(0, "profiles/r3b")
from simlib import world_bound, closest_dist, line_dist

it = int(sys.argv[1]); h = float(sys.argv[2]); ncell = int(sys.argv[3])
D = np.load(f"/tmp/c2_it{it}.npz")
R = float(D["R"])
bs, be, br = D["bs"].astype(np.float64), D["be"].astype(np.float64), D["br"].astype(np.float64)
so, sp, sd, st = D["so"].astype(np.float64), D["sp"].astype(np.float64), D["sd"].astype(np.float64), D["st"].astype(np.float64)
maxd = R + br.max()
E = maxd * 1.001 + 1e-5
glo = np.minimum(so.min(0), sp.min(0)) - E
ghi = np.maximum(so.max(0), sp.max(0)) + E
G = np.ceil((ghi - glo) / h).astype(int)
print("grid", G, "cells", G.prod(), "maxd", maxd)
bv = be - bs; bl = np.linalg.norm(bv, axis=1); bu = bv / bl[:, None]
blo, bhi = world_bound(bs, be, br)
# clip each beam LINE to the grid box -> param range [ta, tb] (extension included)
inv = 1.0 / np.where(bu == 0, 1e-30, bu)
a = (glo - bs) * inv; b = (ghi - bs) * inv
ta = np.minimum(a, b).max(1); tb = np.maximum(a, b).min(1)
# segment-only variant: [0, bl]
major = np.abs(bu).argmax(1)

def beams_in_cell(c, ext=True):
    """beams whose capsule slab-rectangle covers cell c (i, j, k)."""
    lo_c = glo + np.array(c) * h; hi_c = lo_c + h
    t0 = ta if ext else np.zeros_like(ta)
    t1 = tb if ext else bl
    ok = t1 > t0
    # param range of the line inside slab [lo_c[m] - E, hi_c[m] + E] along the major axis m
    m = major
    idx = np.arange(len(bs))
    om, um = bs[idx, m], bu[idx, m]
    sa = (lo_c[m] - E - om) / um; sb = (hi_c[m] + E - om) / um
    s0 = np.maximum(np.minimum(sa, sb), t0); s1 = np.minimum(np.maximum(sa, sb), t1)
    ok &= s1 >= s0
    p0 = bs + bu * s0[:, None]; p1 = bs + bu * s1[:, None]
    pl = np.minimum(p0, p1) - E; ph = np.maximum(p0, p1) + E
    ok &= np.all((pl <= hi_c) & (ph >= lo_c), axis=1)
    return np.nonzero(ok)[0]

def pieces_in_cell(c):
    lo_c = glo + np.array(c) * h - 1e-6; hi_c = lo_c + h + 2e-6
    d = sp - so
    inv = 1.0 / np.where(d == 0, 1e-30, d)
    a = (lo_c - so) * inv; b = (hi_c - so) * inv
    tn = np.maximum(np.minimum(a, b).max(1), 0); tf = np.minimum(np.maximum(a, b).min(1), 1)
    return np.nonzero(tn <= tf)[0]

rng = np.random.default_rng(3)
# sample cells weighted by segment presence: pick random segment points
tot = dict(cells=0, pieces=0, slots=0, entries=0, entries_noext=0, tests=0, queued=0, contrib_owned=0, queued_noext=0)
t0 = time.time()
for _ in range(ncell):
    si = rng.integers(len(so)); u = rng.random()
    pt = so[si] + (sp[si] - so[si]) * u
    c = tuple(np.floor((pt - glo) / h).astype(int))
    P = pieces_in_cell(c); pieces_all = P; Bi = beams_in_cell(c); Bn = beams_in_cell(c, ext=False)
    npk = (len(P) + 63) // 64
    tot["cells"] += 1; tot["pieces"] += len(P); tot["slots"] += npk * 64 * len(Bi)
    tot["entries"] += len(Bi); tot["entries_noext"] += len(Bn); tot["tests"] += len(P) * len(Bi)
    if len(P) == 0 or len(Bi) == 0:
        continue
    w = 1.0
    if len(P) > 512:  # hot cell (near the pinhole): subsample the pieces, scale the counts
        w = len(P) / 512; P = rng.choice(P, 512, replace=False)
    L = np.repeat(P, len(Bi)); Bb = np.tile(Bi, len(P))
    A = sp[L] - so[L]; au = A / np.linalg.norm(A, axis=1)[:, None]
    ld = line_dist(so[L], au, bs[Bb], bu[Bb])
    q = ld <= maxd * 1.0001 + 1e-4
    tot["queued"] += w * int(q.sum())
    tot["queued_noext"] += w * int((q & np.isin(Bb, Bn)).sum())
    L, Bb = L[q], Bb[q]
    # reference contribution + ownership by the cell of pA (recompute pA)
    ok, dist = closest_dist(so[L], sp[L], bs[Bb], be[Bb])
    a_ = (blo[Bb] - so[L]) / np.where(sd[L] == 0, 1e-30, sd[L]); b_ = (bhi[Bb] - so[L]) / np.where(sd[L] == 0, 1e-30, sd[L])
    tn_ = np.minimum(a_, b_).max(1); tf_ = np.maximum(a_, b_).min(1)
    hit = (tn_ <= tf_) & (tn_ < st[L]) & (tf_ > 0)
    con = ok & hit & (dist < maxd)
    tot["contrib_owned"] += w * int(con.sum())  # pairs present in this cell (not yet deduplicated)
    # ownership: the cell of the reference's pA (approximated by the line-line closest point, clamped)
    A = sp[L] - so[L]; ma = np.linalg.norm(A, axis=1); au = A / ma[:, None]
    w0 = so[L] - bs[Bb]; bb = (au * bu[Bb]).sum(1); dd = (au * w0).sum(1); ee = (bu[Bb] * w0).sum(1)
    den = np.maximum(1 - bb * bb, 1e-12); tq = np.clip((bb * ee - dd) / den, 0, ma)
    pa = so[L] + au * tq[:, None]
    own = np.all(np.floor((pa - glo) / h).astype(int) == np.array(c), axis=1)
    tot["contrib_own"] = tot.get("contrib_own", 0) + w * int((con & own).sum())
    tot["w_slots"] = tot.get("w_slots", 0) + (npk * 64 * len(Bi)) / max(len(pieces_all), 1)
    tot["w_queued"] = tot.get("w_queued", 0) + w * int(q.sum()) / max(len(pieces_all), 1)
    tot["w_stage"] = tot.get("w_stage", 0) + npk * len(Bi) / 64.0 / max(len(pieces_all), 1)
print("it", it, "h", h, "cells", ncell, "time %.0f" % (time.time() - t0))
n = tot["cells"]
print("per cell: pieces %.0f entries %.0f (segment-only %.0f) slots %.0f tests %.0f queued %.0f contrib_present %.0f" % (
    tot["pieces"] / n, tot["entries"] / n, tot["entries_noext"] / n, tot["slots"] / n, tot["tests"] / n, tot["queued"] / n, tot["contrib_owned"] / n))
segl = np.linalg.norm(sp - so, axis=1).sum()
npieces = np.abs(sp - so).sum() / h + len(so)  # cells crossed ~ sum |d_i| / h + 1 per segment
print("total pieces ~%.3gM  est. total lane slots %.3gG  queued %.3gG  tile stagings %.3gM  owned/present %.3f" % (
    npieces / 1e6, tot["w_slots"] / n * npieces / 1e9, tot["w_queued"] / n * npieces / 1e9, tot["w_stage"] / n * npieces / 1e6,
    tot["contrib_own"] / tot["contrib_owned"]))
print("slots/queued %.2f tests/queued %.2f contrib/queued %.3f" % (tot["slots"] / tot["queued"], tot["tests"] / tot["queued"], tot["contrib_owned"] / tot["queued"]))
