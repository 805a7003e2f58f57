"""The C2 film is the same bits on every run and whatever the number of contexts (VERDICT r3,
"next round" item 5).

The reference adds a pixel's terms in one fixed order (photonbeam.cpp:477-504: one thread per 16x16
tile, the pixel's path depths in order).  libbre's film path has no float atomics and no
order-dependent hardware step left:
* per segment, the exact stage's ranks come from commutative LDS ORs (bre_gather.hip
  accumulate_batch) and each segment adds its pairs in queue order, the subtrees in root order;
* per pixel, the segments are stably sorted by pixel and one thread adds a pixel's segments in the
  caller's (depth) order (bre_sort.hip launch_pixel_compose);
* per iteration, bench.py's SceneWorkload adds each iteration's image to the one film in iteration
  order, whichever of its contexts (streams) rendered it.
So the whole 16-iteration C2 render (512x512, 1M photons per iteration, the bench's own flow and
options) must be bit-identical across two runs with the two-context pipeline and against a run with
one context."""
import importlib
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _render(n_ctx):
    import torch

    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    bench = importlib.import_module("bench")
    bre = importlib.import_module("beam-radiance-estimate-pbrt_amd")
    dmod = importlib.import_module("beam-radiance-estimate-pbrt_amd.dist")
    args = bench.parse(["--steps", "16", "--warmup", "0"])  # C2: 512x512, 1M photons, 16 iterations
    dev = torch.device("cuda", 0)
    # the bench's own film: packet-class planes (bench.film_classes), as its contexts are set up
    frame = dmod.ShardedFrame(args.width, args.height, 0, 1, device=dev, packets=True,
                              classes=bench.film_classes(args))
    ctxs = [bench.make_context(bre, args, dev) for _ in range(n_ctx)]
    prev = torch.cuda.current_stream()
    torch.cuda.set_stream(ctxs[0][1])
    try:
        wl = bench.SceneWorkload(args, bre, ctxs, frame, 0, 1)
        n = 0
        for k in range(args.steps):
            n += wl.step(k, None, scratch=False)
        wl.finish()
        torch.cuda.synchronize()
        film = frame.resolve().cpu().numpy().copy()
    finally:
        torch.cuda.set_stream(prev)
        for c, _ in ctxs:
            c.close()
    return film, n


@pytest.mark.timeout(300)
def test_c2_film_bit_identical_across_runs_and_contexts():
    a, na = _render(2)
    b, nb = _render(2)
    c, nc = _render(1)
    assert na == nb == nc and na > 5_000_000  # ~0.6M segments per iteration
    assert float(a.sum()) > 0 and np.isfinite(a).all()
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), "two pipelined runs differ"
    assert np.array_equal(a.view(np.uint32), c.view(np.uint32)), "one vs two contexts differ"
