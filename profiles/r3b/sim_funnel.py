"""Filter funnel of the production tile kernel on real C2 data, sampled packets (CPU model).
usage: python profiles/r3b/sim_funnel.py IT NPACK [margin_scale ...]"""
import sys, time, numpy as np
sys.path.insert(0, "profiles/r3b")
from simlib import hilbert_keys, quant, world_bound, ray_box, closest_dist, line_dist

it = int(sys.argv[1]); npk = int(sys.argv[2])
D = np.load(f"/tmp/c2_it{it}.npz")
R = float(D["R"])
bs, be, br = D["bs"].astype(np.float64), D["be"].astype(np.float64), D["br"].astype(np.float64)
so, sp, sd, st, dep = D["so"].astype(np.float64), D["sp"].astype(np.float64), D["sd"].astype(np.float64), D["st"].astype(np.float64), D["sdep"]
# beam tree order: Hilbert 6-D of (start, end)
pts = np.concatenate([bs, be]); lo, hi = pts.min(0), pts.max(0)
kb = hilbert_keys(np.concatenate([quant(bs, lo, hi), quant(be, lo, hi)], 1))
ob = np.argsort(kb, kind="stable")
bs, be, br = bs[ob], be[ob], br[ob]
blo, bhi = world_bound(bs, be, br)
nb = len(bs); T = (nb + 63) // 64
pad = T * 64 - nb
tlo = np.concatenate([blo, np.full((pad, 3), np.inf)]).reshape(T, 64, 3).min(1)
thi = np.concatenate([bhi, np.full((pad, 3), -np.inf)]).reshape(T, 64, 3).max(1)
bvec = be - bs; bmag = np.linalg.norm(bvec, axis=1); bu = bvec / np.where(bmag > 0, bmag, 1)[:, None]
# tile axis lines (mean start -> mean end) and radius rho: every beam LINE, clipped to the region
# R = segment bounds + maxd, lies within rho of the axis line (convexity: check the clip end points)
Rlo = np.minimum(D["so"].min(0), D["sp"].min(0)) - 2 * R - 1e-4
Rhi = np.maximum(D["so"].max(0), D["sp"].max(0)) + 2 * R + 1e-4
padn = T * 64 - nb
S_ = np.concatenate([bs, np.repeat(bs[-1:], padn, 0)]).reshape(T, 64, 3)
E_ = np.concatenate([be, np.repeat(be[-1:], padn, 0)]).reshape(T, 64, 3)
U_ = np.concatenate([bu, np.repeat(bu[-1:], padn, 0)]).reshape(T, 64, 3)
ax0 = S_.mean(1); ax1 = E_.mean(1); axd = ax1 - ax0; axd /= np.linalg.norm(axd, axis=1, keepdims=True)
invu = 1.0 / np.where(U_ == 0, 1e-30, U_)
la = (Rlo - S_) * invu; lb = (Rhi - S_) * invu
tin = np.minimum(la, lb).max(2); tout = np.maximum(la, lb).min(2)
def dist_axis(P):
    w = P - ax0[:, None, :]
    return np.linalg.norm(np.cross(w, axd[:, None, :]), axis=2)
Pin = S_ + U_ * tin[..., None]; Pout = S_ + U_ * tout[..., None]
valid = tout > tin
rho = np.where(valid, np.maximum(dist_axis(Pin), dist_axis(Pout)), 0).max(1)
print("tile rho median %.3f p90 %.3f" % tuple(np.percentile(rho, [50, 90])))
def group_axis(G):
    # axis / rho over G consecutive tiles (a subtree of G leaves)
    TG = T // G
    Sg = S_[:TG * G].reshape(TG, G * 64, 3); Eg = E_[:TG * G].reshape(TG, G * 64, 3); Ug = U_[:TG * G].reshape(TG, G * 64, 3)
    a0 = Sg.mean(1); a1 = Eg.mean(1); ad = a1 - a0; ad /= np.linalg.norm(ad, axis=1, keepdims=True)
    iu = 1.0 / np.where(Ug == 0, 1e-30, Ug)
    l1 = (Rlo - Sg) * iu; l2 = (Rhi - Sg) * iu
    ti = np.minimum(l1, l2).max(2); to = np.maximum(l1, l2).min(2)
    def da(P):
        return np.linalg.norm(np.cross(P - a0[:, None, :], ad[:, None, :]), axis=2)
    rg = np.where(to > ti, np.maximum(da(Sg + Ug * ti[..., None]), da(Sg + Ug * to[..., None])), 0).max(1)
    return a0, ad, rg
GA = {G: group_axis(G) for G in (2, 4)}
for G in (2, 4):
    print("group %d rho median %.3f" % (G, np.median(GA[G][2])))
# segment order: Hilbert 6-D of (o, p)
pts = np.concatenate([so, sp]); lo, hi = pts.min(0), pts.max(0)
ks = hilbert_keys(np.concatenate([quant(so, lo, hi), quant(sp, lo, hi)], 1))
os_ = np.argsort(ks, kind="stable")
so, sp, sd, st, dep = so[os_], sp[os_], sd[os_], st[os_], dep[os_]
ns = len(so); P = ns // 64
rng = np.random.default_rng(1)
pk = rng.choice(P, npk, replace=False)
maxd = R + br  # per beam
scales = [float(x) for x in sys.argv[3:]] or [1.0]
tot = {}
def add(k, v): tot[k] = tot.get(k, 0) + v
t0 = time.time()
for pi in pk:
    sl = slice(pi * 64, pi * 64 + 64)
    o, p, d, tm = so[sl], sp[sl], sd[sl], st[sl]
    A = p - o; ma = np.linalg.norm(A, axis=1); au = A / np.where(ma > 0, ma, 1)[:, None]
    inv = 1.0 / np.where(d == 0, 1e-30, d)
    hit = ray_box(o, inv, tm, tlo, thi)            # (64, T)
    vis = np.nonzero(hit.any(0))[0]
    add("packets", 1); add("primary_packets", int((dep[sl] == 0).mean() > 0.5))
    add("tiles_visited", len(vis))
    # packet bundle (make_bundle)
    co = o.mean(0); su = au.sum(0); cu = su / np.linalg.norm(su)
    def perp(x):
        return np.linalg.norm(np.cross(x - co, cu), axis=-1)
    omax = np.abs(np.concatenate([o, p])).max()
    cm = np.abs(co).max()
    delta = max(perp(o).max(), perp(p).max()) * 1.0001 + 1e-5 * (omax + cm) + 1e-6
    q = o + d * tm[:, None]
    gb = max(perp(o).max(), perp(q).max()) * 1.0001 + 1e-5 * (max(omax, np.abs(q).max()) + cm) + 1e-6
    so_ = ((o - co) * cu).sum(1); sq = ((q - co) * cu).sum(1)
    s0, s1 = min(so_.min(), sq.min()) - 1e-5, max(so_.max(), sq.max()) + 1e-5
    idx = (vis[:, None] * 64 + np.arange(64)[None, :]).ravel()
    idx = idx[idx < nb]
    # bundle_far
    tvec = bs[idx] - co
    n = np.cross(cu, bu[idx]); nn = (n * n).sum(1)
    tn = np.abs((tvec * n).sum(1)); tl = np.abs(tvec).sum(1)
    bmax = np.abs(bs[idx]).max(1)
    mag = omax + bmax + 10 * tl + maxd[idx] + 1; eps = 1e-5 * mag + 1e-6
    far = (nn >= 1e-2) & ((tn - 1e-6 * tl) > ((maxd[idx] + delta) * 1.0001 + 2 * eps) * (np.sqrt(nn) * 1.000001 + 1e-6))
    # bundle_box_miss: segment co + s cu, s in [s0, s1] vs box grown by gb
    c0 = co + cu * s0; dd = cu * (s1 - s0)
    invc = 1.0 / np.where(dd == 0, 1e-30, dd)
    a = (blo[idx] - gb - c0) * invc; b = (bhi[idx] + gb - c0) * invc
    tnb = np.maximum(np.minimum(a, b).max(1), 0); tfb = np.minimum(np.maximum(a, b).min(1), 1)
    miss = tnb > tfb
    keep = ~(far | miss)
    def bundle_keep(sel):
        oo, pp, aa, qq = o[sel], p[sel], au[sel], q[sel]
        co_ = oo.mean(0); su_ = aa.sum(0); cu_ = su_ / np.linalg.norm(su_)
        pr = lambda x: np.linalg.norm(np.cross(x - co_, cu_), axis=-1)
        om_ = np.abs(np.concatenate([oo, pp])).max(); cm_ = np.abs(co_).max()
        de = max(pr(oo).max(), pr(pp).max()) * 1.0001 + 1e-5 * (om_ + cm_) + 1e-6
        g_ = max(pr(oo).max(), pr(qq).max()) * 1.0001 + 1e-5 * (max(om_, np.abs(qq).max()) + cm_) + 1e-6
        so2 = ((oo - co_) * cu_).sum(1); sq2 = ((qq - co_) * cu_).sum(1)
        a0_, a1_ = min(so2.min(), sq2.min()) - 1e-5, max(so2.max(), sq2.max()) + 1e-5
        tv = bs[idx] - co_; nv = np.cross(cu_, bu[idx]); nnv = (nv * nv).sum(1)
        tnv = np.abs((tv * nv).sum(1))
        far_ = (nnv >= 1e-2) & (tnv > (maxd[idx] + de + 2e-5) * np.sqrt(nnv))
        c0_ = co_ + cu_ * a0_; dd_ = cu_ * (a1_ - a0_); ic = 1.0 / np.where(dd_ == 0, 1e-30, dd_)
        aa_ = (blo[idx] - g_ - c0_) * ic; bb_ = (bhi[idx] + g_ - c0_) * ic
        miss_ = np.maximum(np.minimum(aa_, bb_).max(1), 0) > np.minimum(np.maximum(aa_, bb_).min(1), 1)
        return ~(far_ | miss_)
    tix = np.searchsorted(vis, idx // 64)
    # tile-level axis reject: D(C, axis) > rho + delta + maxd
    nax = np.cross(cu, axd[vis]); nnax = np.linalg.norm(nax, axis=1)
    Dax = np.where(nnax > 1e-6, np.abs(((ax0[vis] - co) * nax).sum(1)) / np.maximum(nnax, 1e-12),
                   np.linalg.norm(np.cross(ax0[vis] - co, cu), axis=1))
    skip = Dax > rho[vis] + delta + 2 * R + 1e-4
    kt = np.bincount(tix, weights=keep, minlength=len(vis))
    add("tiles_axis_skip", int(skip.sum())); add("tiles_axis_skip_with_kept", int((skip & (kt > 0)).sum()))
    add("kept_in_skipped", float(kt[skip].sum()))
    for G in (2, 4):
        a0, ad, rg = GA[G]
        gi = vis // G
        gi_ok = gi < len(rg)
        gi = np.minimum(gi, len(rg) - 1)
        nax2 = np.cross(cu, ad[gi]); nn2 = np.linalg.norm(nax2, axis=1)
        D2 = np.where(nn2 > 1e-6, np.abs(((a0[gi] - co) * nax2).sum(1)) / np.maximum(nn2, 1e-12),
                      np.linalg.norm(np.cross(a0[gi] - co, cu), axis=1))
        sk2 = gi_ok & (D2 > rg[gi] + delta + 2 * R + 1e-4)
        add(f"tiles_skip_by_group{G}", int(sk2.sum())); add(f"tiles_skip_by_tile_or_group{G}", int((sk2 | skip).sum()))
    for G in (2, 4):
        kg = np.stack([bundle_keep(slice(g * 64 // G, (g + 1) * 64 // G)) for g in range(G)])  # (G, nidx)
        # lane-steps: per tile max over groups of kept beams (one beam per group per step)
        per = np.stack([np.bincount(tix, weights=kg[g], minlength=len(vis)) for g in range(G)])
        add(f"g{G}_steps", float(per.max(0).sum())); add(f"g{G}_kept", float(kg.sum()))
    add("whole_beamsteps", float(np.bincount(tix, weights=keep, minlength=len(vis)).sum()))
    add("beams_staged", len(idx)); add("beams_kept", int(keep.sum()))
    kidx = idx[keep]
    tile_of = kidx // 64
    # on lanes per kept beam: lanes that hit the beam's TILE box
    onm = hit[:, tile_of]                            # (64, K)
    add("lane_tests", int(onm.sum()))
    kk = np.bincount(np.searchsorted(vis, tile_of), minlength=len(vis))
    add("tiles_zero_kept", int((kk == 0).sum())); add("tiles_le4_kept", int((kk <= 4).sum()))
    add("onlanes_per_tile", int(hit[:, vis].sum()))
    add("scan_steps", int(((kk + 1) // 2).sum()))
    # exact box test and distances for all on pairs
    L, Kb = np.nonzero(onm)
    bi = kidx[Kb]
    bxh = ray_box_pairs = None
    a_ = (blo[bi] - o[L]) * inv[L]; b_ = (bhi[bi] - o[L]) * inv[L]
    tn_ = np.minimum(a_, b_).max(1); tf_ = np.maximum(a_, b_).min(1) * (1 + 6 * 2**-24)
    boxhit = (tn_ <= tf_) & (tn_ < tm[L]) & (tf_ > 0)
    ok, dist = closest_dist(o[L], p[L], bs[bi], be[bi])
    contrib = boxhit & ok & (dist < maxd[bi])
    add("contrib", int(contrib.sum())); add("boxhit_on", int(boxhit.sum()))
    ld = line_dist(o[L], au[L], bs[bi], bu[bi])
    # current prefilter threshold: thr = Ab' + Al'
    o1 = np.abs(o).sum(1); b1 = np.abs(bs[bi]).sum(1); bmx = np.abs(bs[bi]).max(1)
    om = np.maximum(np.abs(o).max(1), np.abs(p).max(1))
    ab_m = 2e-5 * (bmx + 10 * b1) + 2e-6 + 10 * (1e-5 * bmx + 1e-6)
    al_m = 2e-5 * (om[L] + 10 * o1[L]) + 1e-4 * om[L]
    for sc in scales:
        thr = maxd[bi] * 1.0001 + sc * (ab_m + al_m)
        qd = ld <= thr
        add(f"queued@{sc}", int(qd.sum()))
        add(f"queued_contrib@{sc}", int((qd & contrib).sum()))
print("it", it, "R", R, "packets", npk, "time %.1f" % (time.time() - t0))
for k, v in tot.items():
    print(k, v)
Q = tot[f"queued@{scales[0]}"]
print("tiles with 0 kept %.3f, <=4 kept %.3f, on lanes per visited tile %.1f" % (tot["tiles_zero_kept"] / tot["tiles_visited"], tot["tiles_le4_kept"] / tot["tiles_visited"], tot["onlanes_per_tile"] / tot["tiles_visited"]))
print("tile axis reject: %.3f of visited tiles skipped (%.3f of them had kept beams; kept beams dropped %.3f)" % (tot["tiles_axis_skip"] / tot["tiles_visited"], tot["tiles_axis_skip_with_kept"] / max(tot["tiles_axis_skip"], 1), tot["kept_in_skipped"] / tot["beams_kept"]))
print("visited tiles skipped via their group of 2: %.3f, of 4: %.3f (union with tile test: %.3f / %.3f)" % tuple(tot[k] / tot["tiles_visited"] for k in ("tiles_skip_by_group2", "tiles_skip_by_group4", "tiles_skip_by_tile_or_group2", "tiles_skip_by_tile_or_group4")))
print("beam-steps (x64 lanes) per packet: whole %.0f  2 groups %.0f  4 groups %.0f" % (tot["whole_beamsteps"] / npk, tot["g2_steps"] / npk, tot["g4_steps"] / npk))
print("per packet: tiles %.0f staged %.0f kept %.0f (%.3f) lane_tests %.0f scan_steps %.0f" % (
    tot["tiles_visited"] / npk, tot["beams_staged"] / npk, tot["beams_kept"] / npk, tot["beams_kept"] / tot["beams_staged"],
    tot["lane_tests"] / npk, tot["scan_steps"] / npk))
for sc in scales:
    q = tot[f"queued@{sc}"]
    print("margin x%g: tests/queued %.2f  contrib/queued %.3f  lost contrib %d" % (sc, tot["lane_tests"] / q, tot["contrib"] / q, tot["contrib"] - tot[f"queued_contrib@{sc}"]))
