#!/usr/bin/env python3
"""Round-6 study: the tile kernel's dispatch order and tail, from per-wave start / end times (a
BRE_WAVE_TIMES build of bre_gather.hip, profiles/r6/variant_src.sh; s_memrealtime, 100 MHz).
usage (GPU box): BRE_LIBRARY=.../libbre_wt.so python3 profiles/r6/wave_times.py ITER SHARD_RANK SHARD_COUNT
Prints the kernel's span, the span over which its blocks start (dispatch), the tail after the last block
starts, and the fraction of the span's wave-slot time the waves use (1 - idle fraction)."""
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
bre = importlib.import_module("beam-radiance-estimate-pbrt_amd")
sc = importlib.import_module("beam-radiance-estimate-pbrt_amd.scene")

it, rank, count = (int(a) for a in sys.argv[1:4])
scene = sc.cornell_scene(0.05, 0.5, 0.0)
R = bre.beam_radius_at(0.01, 0.5, it)
W = H = 512
with bre.BeamGather(0) as g:
    if count > 1:
        g.set_shard(rank, count, 1, packets=True)
    g.trace_photons(scene, 1_000_000, it, 5, R)
    n = g.camera_pass(scene, W, H, it, 5, True, True)
    film = torch.zeros((W * H, 3), dtype=torch.float32, device="cuda")
    for _ in range(2):  # the second launch is the one read back
        g.gather_camera(R, film)
        g.synchronize()
    m = bre.shard_segments(n, rank, count, 1) if count > 1 else n
    nb = (m + 63) // 64 * 256
    lib = g.lib
    buf = np.zeros(2 * nb, np.uint64)
    lib.bre_study_wave_times.argtypes = [ctypes.c_int64, ctypes.c_void_p]
    assert lib.bre_study_wave_times(nb, buf.ctypes.data) == 0
st, en = buf[:nb].astype(np.float64), buf[nb:].astype(np.float64)
ok = (st > 0) & (en >= st)
st, en = st[ok] * 1e-5, en[ok] * 1e-5  # ms
t0 = st.min()
st, en = st - t0, en - t0
span, last_start = en.max(), st.max()
# concurrency over time: +1 at each start, -1 at each end
ev = np.concatenate([np.stack([st, np.ones_like(st)], 1), np.stack([en, -np.ones_like(en)], 1)])
ev = ev[np.argsort(ev[:, 0], kind="stable")]
conc = np.cumsum(ev[:, 1])
dt = np.diff(ev[:, 0], append=ev[-1, 0])
peak = np.percentile(conc, 99)
busy = float((conc * dt).sum())
below = float(dt[conc < 0.5 * peak].sum())
dur = en - st
print(f"iteration {it} shard {rank}/{count}: waves {ok.sum()} span {span:.2f} ms, blocks start over {last_start:.2f} ms, "
      f"tail after the last start {span - last_start:.2f} ms, concurrency p99 {peak:.0f}, "
      f"slot use {busy / (span * peak):.3f}, time below half the peak {below:.2f} ms, "
      f"wave ms mean {dur.mean():.3f} p99 {np.percentile(dur, 99):.3f} max {dur.max():.3f}")
