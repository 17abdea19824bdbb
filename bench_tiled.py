"""Config C5: 2048x2048 RGB images filtered as overlap-save 256x256 windows (tiling.py) by the
10-stage G=32 image filter; one process per GPU, windows sharded over ranks, no collective in
the data path (gather of the output canvas only with --gather).

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
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # GRR_BENCH_BACKEND=gloo + fewer GPUs than ranks: multi-rank rehearsal on a one-GPU box
    dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
    if world > 1:
        torch.cuda.set_device(dev)
        backend = os.environ.get("GRR_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=dev)
        else:
            torch.distributed.init_process_group(backend)
    import irdu_amd
    from irdu_amd import tiling
    from bench import build_model, synthetic_patches
    irdu_amd.load_native()
    model = build_model(dev)
    _, noisy = synthetic_patches(args.images, seed=2204, h=args.size, w=args.size)
    noisy = noisy.to(dev)
    run = lambda: tiling.tiled_forward(model, noisy, tile=args.tile, halo=args.halo, align=16,  # noqa: E731
                                       micro_batch=args.micro_batch, gather=args.gather)
    run()
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    dt = float(t.item())
    nwin = len(tiling.tile_grid(args.size, args.size, args.tile, args.halo, 16))
    if rank == 0:
        px = args.images * args.size * args.size * args.steps
        print(json.dumps({"metric": "tiled inference MPix/s (output pixels)", "value": round(px / dt / 1e6, 3),
                          "unit": "MPix/s", "n_gpus": world, "ms_per_step": round(dt / args.steps * 1e3, 2),
                          "config": {"workload": f"{args.images} x {args.size}^2 RGB, {args.tile}^2 windows, halo "
                                                 f"{args.halo}, G=32 F=3 S=10 image filter",
                                     "windows_per_image": nwin,
                                     "window_overhead": round(nwin * args.tile ** 2 / args.size ** 2, 3),
                                     "parallelism": f"windows sharded x{world}"}}))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
