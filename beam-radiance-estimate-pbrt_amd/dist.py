"""Multi-GPU decomposition of the gather: image tiles (or packet ranges) across ranks, beams replicated.

The reference's camera pass already works in 16x16 pixel tiles (photonbeam.cpp:345-347, 444-557);
here those tiles are dealt round-robin to the ranks (one process per GPU; libbre's camera pass walks
only the rank's tiles, BRE_OPT_SHARD_RANK / BRE_OPT_SHARD_COUNT).  Every rank holds the whole beam
set (each traces the same photons from the same per-photon PCG32 sequences, photonbeam.cpp:386-389,
so the data path has no communication) and builds its own BVH; each pixel is written by exactly
one rank.  The only exchange is one framebuffer GATHER per written image (photonbeam.cpp:565-584):
every rank packs the pixels of its own tiles into a contiguous band (1/N of the film) and the bands
are gathered to the root over RCCL (backend "nccl") or gloo (CPU tests), which scatters them back
into the full film.  Ownership is disjoint, so the gathered film equals the sum of the ranks'
partial films exactly.

Packet shards (``packets=True``, BRE_OPT_SHARD_MODE 1, the bench's default for strong scaling): every
rank runs the whole camera pass and sorts all segments as one GPU would, then gathers only its
round-robin share of the sorted 64-segment packets (p = rank mod N, ``bre_shard_segments``), so its
packets are exactly the single-GPU packets and every rank gets the same mix of cheap and costly ones (tile shards thin out each rank's bounce segments N-fold and loosen its
packets: 1.5M vs 2.3M estimates/s per GPU at N=8, profiles/r2/explore/explore28-29).  A pixel's
segments may then sit on several ranks: the films are partial sums, combined by one RCCL reduce.

Work-root shards (bench ``--shard-mode roots``, BRE_OPT_SHARD_MODE 2; the frame is built with
``packets=True``): every rank gathers every segment against its share of the BVH work roots, so its
films are partial sums too and take the same reduce.

Packet-class films (``classes=8``, libbre BRE_OPT_FILM_CLASSES; the bench's default): the film is kept
as 8 planes -- plane c takes the surface radiance of the pixels p = c (mod 8) and the gather terms of
the sorted order's packets k = c (mod 8) -- and the image is their sum in class order.  With N ranks
(N dividing 8) rank r computes exactly the planes c = r (mod N), each bit for bit as one GPU computes
it (a segment's sum does not depend on which rank gathers its packet), so one GATHER of the ranks'
planes to the root and the resolve give the one-GPU image bit for bit, where the sum-reduce of partial
films could not (it adds a pixel's terms in another grouping).
"""
from __future__ import annotations

import numpy as np


def tile_pixels(w: int, h: int, rank: int, world: int, tile: int = 16, block: int = 1) -> np.ndarray:
    """Pixel indices (y*w + x) of the tiles owned by `rank` -- the tiles of the blocks of block x block
    tiles whose row-major block index is rank (mod world), as libbre's camera pass deals them
    (BRE_OPT_SHARD_BLOCK) -- tile-major in row-major tile order, row-major inside a tile."""
    ntx = (w + tile - 1) // tile
    nty = (h + tile - 1) // tile
    nbx = (ntx + block - 1) // block
    out = []
    for t in range(ntx * nty):
        tx, ty = t % ntx, t // ntx
        if ((ty // block) * nbx + tx // block) % world != rank:
            continue
        xs = np.arange(tx * tile, min(tx * tile + tile, w))
        ys = np.arange(ty * tile, min(ty * tile + tile, h))
        out.append((ys[:, None] * w + xs[None, :]).ravel())
    return np.concatenate(out).astype(np.int64) if out else np.zeros(0, dtype=np.int64)


class ShardedFrame:
    """Full-resolution RGB accumulation buffer of one rank (only its own tiles are ever written)."""

    def __init__(self, w: int, h: int, rank: int, world: int, device="cpu", tile: int = 16, block: int = 1,
                 packets: bool = False, classes: int = 1, roots: bool = False):
        import torch

        self.w, self.h, self.rank, self.world, self.tile, self.block = w, h, rank, world, tile, block
        # packets=True: PACKET shards (BRE_OPT_SHARD_MODE 1) -- every rank may write every pixel (its
        # range of the sorted segment packets), and the films are SUMMED by one reduce, or, with
        # classes=8 (packet-class films), gathered plane by plane.  roots=True: WORK-ROOT shards
        # (BRE_OPT_SHARD_MODE 2) -- every rank writes partial sums of every pixel in every plane, so only
        # the sum-reduce combines them (libbre refuses class films under root shards as well)
        self.roots = roots
        self.packets = packets or roots
        if classes != 1 and (roots or not packets):
            raise ValueError("packet-class films need packet shards (not tile or work-root shards)")
        self.classes = classes
        self.pixels = np.arange(w * h, dtype=np.int64) if self.packets else tile_pixels(w, h, rank, world, tile, block)
        # with classes: (classes * w * h, 3), plane c = rows [c * w * h, (c + 1) * w * h)
        self.accum = torch.zeros((classes * w * h, 3), dtype=torch.float32, device=device)
        self.device = device
        self._band = None
        if not self.packets:  # the band machinery (also at world 1: a live 1-rank group still runs the gather)
            counts = [tile_pixels(w, h, r, world, tile, block).shape[0] for r in range(world)]
            self.band_len = max(counts)
            self._idx = torch.from_numpy(self.pixels).to(device)
            self._all_idx = [torch.from_numpy(tile_pixels(w, h, r, world, tile, block)).to(device)
                             for r in range(world)]

    @property
    def npix(self) -> int:
        return self.w * self.h

    def band(self):
        """This rank's owned pixels packed into a contiguous (band_len, 3) band (zero padded)."""
        import torch

        band = torch.zeros((self.band_len, 3), dtype=torch.float32, device=self.device)
        band[: self._idx.shape[0]] = self.accum.index_select(0, self._idx)
        return band

    def scatter_bands(self, parts, skip: int | None = None):
        """Write every rank's band (parts[r]) back to its tiles of this frame (rank `skip` left as is)."""
        for r, idx in enumerate(self._all_idx):
            if r != skip:
                self.accum.index_copy_(0, idx, parts[r][: idx.shape[0]].to(self.accum.device))
        return self.accum

    def gather_bands(self, root: int = 0):
        """Tile shards: the ranks' owned-pixel bands gathered to `root` (one collective); the list of
        bands on the root, None elsewhere."""
        import torch
        import torch.distributed as dist

        band = self.band()
        parts = [torch.empty_like(band) for _ in range(self.world)] if self.rank == root else None
        dist.gather(band, gather_list=parts, dst=root)
        return parts

    def gather_to_root(self, root: int = 0):
        """One collective per written image: each rank's band of owned pixels (packed, 1/N of the
        film) is gathered to `root`, which scatters the bands into the full film.  Returns the full
        film on the root (the rank's own partial film elsewhere).  Without a live process group a
        one-rank frame is returned as it is; with one (also of size 1: tests/test_rccl_gpu.py) the
        collective always runs."""
        import torch.distributed as dist

        live = dist.is_available() and dist.is_initialized()
        if self.world == 1 and not live:
            return self.accum
        if self.packets and not self.roots and self.classes > 1 and self.classes % self.world == 0:
            return self._gather_planes(root)
        if self.packets:  # partial films of one image: one sum-reduce to the root
            if dist.get_backend() == "gloo" and self.accum.is_cuda:  # gloo reduces host tensors
                host = self.accum.cpu()
                dist.reduce(host, dst=root, op=dist.ReduceOp.SUM)
                if self.rank == root:
                    self.accum.copy_(host)
            else:
                dist.reduce(self.accum, dst=root, op=dist.ReduceOp.SUM)
            return self.accum
        parts = self.gather_bands(root)
        if self.rank == root:
            self.scatter_bands(parts, skip=root)
        return self.accum

    def owned_planes(self, rank: int | None = None):
        """The class planes rank `rank` (default: this rank) computes: c = rank (mod world)."""
        r = self.rank if rank is None else rank
        return [c for c in range(self.classes) if c % self.world == r]

    def plane(self, c: int):
        n = self.w * self.h
        return self.accum[c * n:(c + 1) * n]

    def _gather_planes(self, root: int):
        """Packet-class films: each rank's own planes (classes / world of them, contiguous) gathered to
        the root, which writes them into its planes -- every plane as the rank that owns it computed it."""
        import torch
        import torch.distributed as dist

        mine = torch.cat([self.plane(c) for c in self.owned_planes()])
        host = dist.get_backend() == "gloo" and mine.is_cuda  # gloo gathers host tensors
        send = mine.cpu() if host else mine
        parts = [torch.empty_like(send) for _ in range(self.world)] if self.rank == root else None
        dist.gather(send, gather_list=parts, dst=root)
        if self.rank == root:
            n = self.w * self.h
            for r, part in enumerate(parts):
                if r == root:
                    continue
                for k, c in enumerate(self.owned_planes(r)):
                    self.plane(c).copy_(part[k * n:(k + 1) * n].to(self.accum.device))
        return self.accum

    def resolve(self):
        """The image of a packet-class film: the planes added in class order (plane 0 + plane 1 + ...,
        the order bre_resolve_classes uses), on the root after gather_to_root(); the film itself without
        classes."""
        if self.classes == 1:
            return self.accum
        out = self.plane(0).clone()
        for c in range(1, self.classes):
            out += self.plane(c)
        return out

    # the round-1 name (a reduce of full frames); kept as an alias of the gather
    reduce_to_root = gather_to_root

    def image(self, iteration: int):
        """L = Ld / (iter + 1)  (photonbeam.cpp:578), on the root after gather_to_root()."""
        return self.resolve() / float(iteration + 1)
