"""Multi-GPU decomposition of the gather: image tiles across ranks, beams replicated.

The reference's camera pass already works in 16x16 pixel tiles (photonbeam.cpp:345-347, 444-557);
here those tiles are dealt round-robin to the ranks (one process per GPU), every rank holds the
whole beam set (regenerated from the same seeds, or broadcast once per pass) and builds its own
BVH, and each pixel is written by exactly one rank.  The only exchange is one framebuffer
reduction per written image (photonbeam.cpp:565-584), an RCCL reduce over xGMI with the "nccl"
backend (gloo in the CPU tests).  Because ownership is disjoint, the reduced image is bit-identical
to a single-rank render: every pixel is x + 0 + ... + 0.
"""
from __future__ import annotations

import numpy as np


def tile_pixels(w: int, h: int, rank: int, world: int, tile: int = 16) -> np.ndarray:
    """Pixel indices (y*w + x) of the tiles owned by `rank`, tile-major, row-major inside a tile."""
    ntx = (w + tile - 1) // tile
    nty = (h + tile - 1) // tile
    out = []
    for t in range(rank, ntx * nty, world):
        tx, ty = t % ntx, t // ntx
        xs = np.arange(tx * tile, min(tx * tile + tile, w))
        ys = np.arange(ty * tile, min(ty * tile + tile, h))
        out.append((ys[:, None] * w + xs[None, :]).ravel())
    return np.concatenate(out).astype(np.int64) if out else np.zeros(0, dtype=np.int64)


class ShardedFrame:
    """Full-resolution RGB accumulation buffer of one rank (zeros outside its tiles)."""

    def __init__(self, w: int, h: int, rank: int, world: int, device="cpu", tile: int = 16):
        import torch

        self.w, self.h, self.rank, self.world = w, h, rank, world
        self.pixels = tile_pixels(w, h, rank, world, tile)
        self.accum = torch.zeros((w * h, 3), dtype=torch.float32, device=device)

    @property
    def npix(self) -> int:
        return self.w * self.h

    def reduce_to_root(self, root: int = 0):
        """One collective per written image: sum the disjoint partial frames onto `root`."""
        import torch.distributed as dist

        if self.world > 1:
            dist.reduce(self.accum, dst=root)
        return self.accum

    def image(self, iteration: int):
        """L = Ld / (iter + 1)  (photonbeam.cpp:578), on the root after reduce_to_root()."""
        return self.accum / float(iteration + 1)
