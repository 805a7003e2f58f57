"""CPU model (round 5): the beam-major scan with the packet's lanes split in G groups, each with its own
bundle line (bbox-centre line, its own delta): a scan step then tests one beam per group at once (group
g's lanes test a beam of group g's kept list), so a tile costs max_g |kept_g| beams of steps instead of
|kept of the whole-packet bundle|.  On real C2 packets (profiles/r5/sim_data.py), per visited tile:
on = lanes whose ray hits the tile box; a group with no lane on keeps nothing.
usage: python profiles/r5/sim_split.py IT NPACK"""
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


def far_bundle(o, p, b0, u, md):
    c_o = 0.5 * (o.min(0) + o.max(0)); c_p = 0.5 * (p.min(0) + p.max(0))
    cu = c_p - c_o; cu /= max(np.linalg.norm(cu), 1e-30)
    X = np.concatenate([o, p])
    delta = np.linalg.norm(np.cross(X - c_o, cu), axis=1).max()
    n = np.cross(cu, u); nl = np.linalg.norm(n, axis=1)
    t = np.abs(((b0 - c_o) * n).sum(1))
    return (nl >= 0.1) & (t / np.maximum(nl, 1e-12) > md + delta)


def lane_far(o, au, b0, u, md):
    """the per-lane scan test (line distance), lanes x beams"""
    n = np.cross(au[:, None, :], u[None, :, :]); nl = np.linalg.norm(n, axis=2)
    t = np.abs(((b0[None] - o[:, None]) * n).sum(2))
    return (nl >= 0.1) & (t / np.maximum(nl, 1e-12) > md[None])


def cost(on, kept):  # the kernel's choice: transposed scan when on * 8 < kept * 6
    return on if on * 8 < kept * 6 else (kept + 1) // 2


GS = (1, 2, 4, 8)
t0 = time.time()
for pi in pk:
    sl = slice(pi * 64, pi * 64 + 64)
    o, p, d, tm = so[sl], sp[sl], sd[sl], st[sl]
    kind = "primary" if (dep[sl] == 0).mean() > 0.5 else "bounce"
    A = p - o; ma = np.linalg.norm(A, axis=1); au = A / np.where(ma > 0, ma, 1)[:, None]
    inv = 1.0 / np.where(d == 0, 1e-30, d)
    hit = ray_box(o, inv, tm, tlo, thi)  # lanes x tiles
    vis = np.nonzero(hit.any(0))[0]
    for tt in vis:
        idx = np.arange(tt * 64, min(tt * 64 + 64, nb))
        b0, u, md = bs[idx], bu[idx], maxd[idx]
        onl = hit[:, tt]
        lf = lane_far(o, au, b0, u, md)  # 64 x nbeams
        useful = int((~lf & onl[:, None]).sum())
        add((kind, "useful"), useful)
        add((kind, "tiles"), 1)
        for G in GS:
            L = 64 // G
            kmax, kall, steps, lanetests = 0, np.zeros(len(idx), bool), 0, 0
            ks = []
            for g in range(G):
                gl = slice(g * L, g * L + L)
                if not onl[gl].any():
                    ks.append(0)
                    continue
                kg = ~far_bundle(o[gl], p[gl], b0, u, md)
                ks.append(int(kg.sum()))
                kall |= kg
            on = int(onl.sum())
            if G == 1:
                steps = cost(on, ks[0])
            else:  # split steps (beam-major, one beam per group per step, two per step for ILP)
                steps = min(cost(on, int(kall.sum())), (max(ks) + 1) // 2)
            add((kind, f"steps{G}"), steps)
            add((kind, f"union{G}"), int(kall.sum()) if G > 1 else ks[0])
            add((kind, f"ustep{G}"), cost(on, int(kall.sum()) if G > 1 else ks[0]))
            add((kind, f"kept{G}"), sum(ks))
print("it", it, "R %.5f" % R, "packets", npk, "time %.1f s" % (time.time() - t0))
for kind in ("primary", "bounce"):
    n = tot.get((kind, "tiles"), 0)
    if not n:
        continue
    print(f"{kind}: tiles {n}, useful lane pairs/tile {tot[(kind, 'useful')] / n:.1f};",
          "  ".join(f"G{G}: steps/tile {tot[(kind, f'steps{G}')] / n:.2f} kept/tile {tot[(kind, f'kept{G}')] / n:.1f} "
                    f"union/tile {tot[(kind, f'union{G}')] / n:.1f} union steps/tile {tot[(kind, f'ustep{G}')] / n:.2f}"
                    for G in GS))
