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

Windows are batched through the model (``micro_batch`` windows per launch).  With N ranks
each rank filters a contiguous share of the windows (sharding.shard_range, no collective);
``gather=True`` sums the disjoint per-rank canvases with one all-reduce.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

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


@torch.no_grad()
def tiled_forward(model, img: torch.Tensor, tile: int = 256, halo: int = 32, align: int = 16,
                  micro_batch: int = 32, out_channels: Optional[int] = None, gather: bool = True) -> torch.Tensor:
    """Filter img [B,C,H,W] window by window; returns the [B,Cout,H,W] output canvas.

    Multi-rank: every rank must call this with the same image; each filters its share of the
    windows.  gather=False returns the rank's partial canvas (zeros outside its cores)."""
    b, c, h, w = img.shape
    th, tw = min(tile, h), min(tile, w)
    wins = tile_grid(h, w, tile, halo, align)
    rank, world = sharding.world()
    s, e = sharding.shard_range(len(wins), rank, world)
    mine = wins[s:e]
    cout = out_channels if out_channels is not None else c
    canvas = torch.zeros((b, cout, h, w), dtype=img.dtype, device=img.device)
    for i in range(0, len(mine), micro_batch):
        chunk = mine[i:i + micro_batch]
        x = torch.cat([img[:, :, wr:wr + th, wc:wc + tw] for wr, wc, *_ in chunk]).contiguous()
        y = model(x)
        for j, (wr, wc, r0, r1, c0, c1) in enumerate(chunk):
            canvas[:, :, r0:r1, c0:c1] = y[j * b:(j + 1) * b, :, r0 - wr:r1 - wr, c0 - wc:c1 - wc]
    if gather and world > 1:
        torch.distributed.all_reduce(canvas)
    return canvas
