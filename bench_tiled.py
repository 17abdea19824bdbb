"""Config C5: 2048x2048 RGB images filtered as overlap-save 256x256 windows (tiling.py) by the
10-stage G=32 image filter; one process per GPU, (image, window) units sharded over ranks -- whole
images first -- with no collective in the data path (--gather: rank 0 also receives every rank's
packed cores, each output pixel once).

    python bench_tiled.py [--images 2] [--size 2048] [--tile 256] [--halo 32] [--micro-batch 64]

Prints one JSON line: MPix/s of output image pixels (whole job), window overhead factor.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=2)
    ap.add_argument("--size", type=int, default=2048)
    ap.add_argument("--tile", type=int, default=256)
    ap.add_argument("--halo", type=int, default=32)
    ap.add_argument("--micro-batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--gather", action="store_true")
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one process per GPU; spawned when not under torchrun)")
    ap.add_argument("--dry-run", action="store_true", help="launcher check: ranks report and exit (no HIP)")
    args = ap.parse_args()
    import benchlib
    world, rank, local = benchlib.join_or_spawn(args.gpus, dry_run=args.dry_run)
    if args.dry_run:
        benchlib.dry_run_report(world, rank, local)
        return
    dev = benchlib.init(world, local)
    ranks = benchlib.check_ranks(world, dev)     # every rank in the group, over the data backend
    import irdu_amd
    from irdu_amd import tiling
    from bench import TRAINED, build_model, synthetic_patches
    irdu_amd.load_native()
    trained = os.path.exists(TRAINED)
    model = build_model(dev, trained=trained)
    _, noisy = synthetic_patches(args.images, seed=2204, h=args.size, w=args.size)
    noisy = noisy.to(dev)
    run = lambda: tiling.tiled_forward(model, noisy, tile=args.tile, halo=args.halo, align=16,  # noqa: E731
                                       micro_batch=args.micro_batch, gather="rank0" if args.gather else "none")
    run()
    benchlib.barrier(world, dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    benchlib.barrier(world, dev)
    dt = benchlib.max_over_ranks(time.perf_counter() - t0, world, dev)
    nwin = len(tiling.tile_grid(args.size, args.size, args.tile, args.halo, 16))
    parity = None
    if world == 1:
        # tiled vs the whole image in one launch (image 0): the halo's effect on the output
        with torch.no_grad():
            tiled = run()[:1]
            whole = model(noisy[:1])
        ref = whole.abs().max().item()
        parity = {"image": "0 of the batch", "max_abs_err_vs_whole": (tiled - whole).abs().max().item(),
                  "rel_err_vs_whole": (tiled - whole).abs().max().item() / ref,
                  "weights": "trained fixture" if trained else "reference init"}
    if rank == 0:
        px = args.images * args.size * args.size * args.steps
        print(json.dumps({"metric": "tiled inference MPix/s (output pixels)", "value": round(px / dt / 1e6, 3),
                          "unit": "MPix/s", "n_gpus": world, "ms_per_step": round(dt / args.steps * 1e3, 2),
                          "config": {"workload": f"{args.images} x {args.size}^2 RGB, {args.tile}^2 windows, halo "
                                                 f"{args.halo}, G=32 F=3 S=10 image filter",
                                     "windows_per_image": nwin,
                                     "window_overhead": round(nwin * args.tile ** 2 / args.size ** 2, 3),
                                     "weights": "tests/golden/msgf_trained_g32_s10.safetensors" if trained
                                     else "reference init",
                                     "parallelism": f"(image, window) units sharded x{world}, "
                                                    + ("cores gathered to rank 0" if args.gather else "no collective")},
                          "tiled_vs_whole": parity, **(ranks if world > 1 else {})}), flush=True)
    benchlib.finish(world)


if __name__ == "__main__":
    main()
