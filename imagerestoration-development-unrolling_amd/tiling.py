"""Overlap-save tiled inference for large images (config C5: 2048x2048, 256x256 tiles).

The reference evaluates whole images padded to a multiple of 16 (scripts_v2/...sigma25.py:
249-262).  For images larger than one launch should hold, the image is cut into windows of
``tile`` pixels whose central ``core = tile - 2*halo`` region is kept (overlap-save):

* cores partition the image; each window is its core grown by ``halo`` on every side and
  shifted (not padded) to stay inside the image, so a window touching the image border has
  the image border as its own border — the model's replicate padding there is exactly the
  whole-image one;
* window origins are multiples of ``align`` (16 for the 4-level v1.0 model, 2 for the
  two-scale filter), so every 2x2 pooling grid inside a window lines up with the image's;
* inside a window a core pixel sees the same inputs as in the whole image as long as
  ``halo`` covers the model's receptive field; the unrolled solver's influence decays
  geometrically with distance, so the result converges to the whole-image one as ``halo``
  grows (tests/test_gpu_tiling.py measures it).

Windows are batched through the model (``micro_batch`` windows per launch).  The work units are
(image, window) pairs in image-major order; with N ranks each rank filters a contiguous share of them
(sharding.shard_range), so a batch of at least N images shards whole images and a single image
shards its windows -- no collective in the data path either way.  Each rank
returns its own cores; ``gather="rank0"`` additionally sends every rank's cores -- only the cores,
each output pixel once -- to rank 0, which assembles the full canvas.
"""
from __future__ import annotations

from typing import List, Optional, Tuple, Union

import torch

from . import sharding

Window = Tuple[int, int, int, int, int, int]   # (wr, wc, r0, r1, c0, c1): window origin + core box


def _axis(n: int, tile: int, halo: int, align: int) -> List[Tuple[int, int, int]]:
    """(window start, core start, core end) along one axis."""
    if n <= tile:
        return [(0, 0, n)]
    core = tile - 2 * halo
    out = []
    for r0 in range(0, n, core):
        r1 = min(r0 + core, n)
        ws = min(max(r0 - halo, 0), n - tile)
        ws -= ws % align
        out.append((ws, r0, r1))
    return out


def tile_grid(h: int, w: int, tile: int = 256, halo: int = 32, align: int = 16) -> List[Window]:
    """Windows covering an h x w image; cores partition it, windows lie inside it."""
    if tile % align or halo % align or (tile - 2 * halo) <= 0:
        raise ValueError(f"tile ({tile}) and halo ({halo}) must be multiples of align ({align}), tile > 2*halo")
    for n in (h, w):
        if n > tile and n % align:
            raise ValueError(f"image side {n} must be a multiple of align ({align}) when it exceeds the tile")
    return [(wr, wc, r0, r1, c0, c1) for wr, r0, r1 in _axis(h, tile, halo, align)
            for wc, c0, c1 in _axis(w, tile, halo, align)]


def rank_units(b: int, n_windows: int, rank: int, world: int) -> List[Tuple[int, int]]:
    """This rank's (image, window) units: a contiguous share of the image-major enumeration."""
    s, e = sharding.shard_range(b * n_windows, rank, world)
    return [divmod(u, n_windows) for u in range(s, e)]


def _core_numel(units, wins, cout: int) -> int:
    return sum(cout * (wins[wi][3] - wins[wi][2]) * (wins[wi][5] - wins[wi][4]) for _, wi in units)


@torch.no_grad()
def tiled_forward(model, img: torch.Tensor, tile: int = 256, halo: int = 32, align: int = 16,
                  micro_batch: int = 32, out_channels: Optional[int] = None,
                  gather: Union[bool, str] = "none") -> Optional[torch.Tensor]:
    """Filter img [B,C,H,W] window by window; returns the [B,Cout,H,W] output canvas.

    One rank: the whole canvas.  Several ranks (every rank calls this with the same image):
    ``gather="none"`` (or False) returns the rank's canvas holding its own cores (zeros elsewhere),
    with no communication; ``gather="rank0"`` (or True) returns the full canvas on rank 0 and None on
    the other ranks, after one gather of the packed cores."""
    mode = {True: "rank0", False: "none"}.get(gather, gather)
    if mode not in ("none", "rank0"):
        raise ValueError(f"gather must be 'none' or 'rank0' (got {gather!r})")
    b, c, h, w = img.shape
    th, tw = min(tile, h), min(tile, w)
    wins = tile_grid(h, w, tile, halo, align)
    rank, world = sharding.world()
    mine = rank_units(b, len(wins), rank, world)
    cout = out_channels if out_channels is not None else c
    canvas = torch.zeros((b, cout, h, w), dtype=img.dtype, device=img.device)
    for i in range(0, len(mine), micro_batch):
        chunk = mine[i:i + micro_batch]
        x = torch.cat([img[bi:bi + 1, :, wins[wi][0]:wins[wi][0] + th, wins[wi][1]:wins[wi][1] + tw]
                       for bi, wi in chunk]).contiguous()
        y = model(x)
        for j, (bi, wi) in enumerate(chunk):
            wr, wc, r0, r1, c0, c1 = wins[wi]
            canvas[bi, :, r0:r1, c0:c1] = y[j, :, r0 - wr:r1 - wr, c0 - wc:c1 - wc]
    if world == 1 or mode == "none":
        return canvas
    return _gather_cores(canvas, wins, b, cout, rank, world)


def _gather_cores(canvas: torch.Tensor, wins, b: int, cout: int, rank: int, world: int) -> Optional[torch.Tensor]:
    """Rank 0 receives every rank's cores (packed, padded to the largest share) and fills its canvas."""
    import torch.distributed as dist
    sizes = [_core_numel(rank_units(b, len(wins), r, world), wins, cout) for r in range(world)]
    n = max(sizes)
    packed = canvas.new_zeros(n)
    off = 0
    for bi, wi in rank_units(b, len(wins), rank, world):
        _, _, r0, r1, c0, c1 = wins[wi]
        k = cout * (r1 - r0) * (c1 - c0)
        packed[off:off + k] = canvas[bi, :, r0:r1, c0:c1].reshape(-1)
        off += k
    bufs = [torch.empty_like(packed) for _ in range(world)] if rank == 0 else None
    dist.gather(packed, bufs, dst=0)
    if rank != 0:
        return None
    for r in range(1, world):
        off = 0
        for bi, wi in rank_units(b, len(wins), r, world):
            _, _, r0, r1, c0, c1 = wins[wi]
            k = cout * (r1 - r0) * (c1 - c0)
            canvas[bi, :, r0:r1, c0:c1] = bufs[r][off:off + k].view(cout, r1 - r0, c1 - c0)
            off += k
    return canvas
