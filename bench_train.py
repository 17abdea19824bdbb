"""Training-step benchmark (config C4 family): forward + HIP reverse sweep + Adam (+ RCCL
gradient all-reduce when launched with torchrun), on synthetic sigma=25 patches resident in HBM.

    python bench_train.py [--model abstract|msgf] [--size 256] [--batch 8] [--stages 10]
                          [--steps 5] [--warmup 2] [--breakdown]

Not the headline metric (bench.py is); prints one JSON line with training MPix/s (input
pixels of the optimisation step per second, whole job) and the per-kernel-kind time of the
HIP launches (forward and reverse), timed with HIP events on their launch stream.
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

D_ARGS = dict(dims=[48, 96, 192, 384], hidden_dims=[96, 192, 384, 768], nsubnets=[1, 1, 1, 1],
              ngraphs=[8, 16, 16, 32], num_blocks=[4, 6, 6, 8], num_blocks_out=4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", choices=["abstract", "msgf"], default="abstract")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--batch", type=int, default=8, help="patches per GPU")
    ap.add_argument("--stages", type=int, default=10)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--aux-losses", action="store_true", help="add the enc-dec / latent-perturbation losses")
    ap.add_argument("--breakdown", action="store_true")
    ap.add_argument("--fused-fts", type=str, default=None,
                    help="comma list of F that use the one-pass term reverses (default: all instances)")
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
    from irdu_amd import kernels as K
    from irdu_amd import training as T
    from bench import synthetic_patches
    irdu_amd.load_native()
    if args.fused_fts is not None:
        K.FUSED_TERM_FTS = tuple(int(v) for v in args.fused_fts.split(",") if v)
    torch.manual_seed(2204)
    if args.model == "abstract":
        model = irdu_amd.AbtractMultiScaleGraphFilter(3, 3, n_cgd_iters=args.stages, **D_ARGS)
        desc = f"AbtractMultiScaleGraphFilter v1.0 dims {D_ARGS['dims']} ngraphs {D_ARGS['ngraphs']}"
    else:
        model = irdu_amd.MultiScaleGraphFilter(3, 3, ngraphs=32, n_cgd_iters=args.stages)
        desc = "MultiScaleGraphFilter G=32 F=3 (v13 feature CNN)"
    w = 0.1 if args.aux_losses else 0.0
    tr = T.Trainer(model, {"loss02_weight": w, "loss03_weight": 5 * w}, dev)
    clean, noisy = synthetic_patches(args.batch, seed=2204 + rank, h=args.size, w=args.size)
    noisy_hwc = noisy.permute(0, 2, 3, 1).contiguous().to(dev)
    clean_hwc = clean.permute(0, 2, 3, 1).contiguous().to(dev)

    def barrier():
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        tr.step(noisy_hwc, clean_hwc)
    barrier()
    timer = K.LaunchTimer()
    K.set_timer(timer)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = tr.step(noisy_hwc, clean_hwc)
    barrier()
    dt = time.perf_counter() - t0
    K.set_timer(None)
    kern = timer.summary()
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    dt = float(t.item())
    if rank == 0:
        px = world * args.batch * args.size * args.size * args.steps
        hip_ms = sum(v["total_ms"] for v in kern.values()) / args.steps
        res = {"metric": "training MPix/s (fwd + HIP reverse + Adam)", "value": round(px / dt / 1e6, 4),
               "unit": "MPix/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": round(dt / args.steps * 1e3, 2), "higher_is_better": True, "scaling": "weak",
               "dtype": "f32", "data": "synthetic",
               "config": {"workload": f"{desc}, S={args.stages}, {args.size}x{args.size} RGB sigma=25",
                          "per_gpu_batch": args.batch, "aux_losses": args.aux_losses,
                          "parallelism": f"data parallel x{world}, bucketed RCCL grad all-reduce"},
               "loss": loss, "hip_kernel_ms_per_step": round(hip_ms, 2),
               "peak_mem_gb": round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 1),
               "kernel_ms_per_step": {k: round(v["total_ms"] / args.steps, 3) for k, v in kern.items()}}
        if args.breakdown:
            for k, v in sorted(kern.items(), key=lambda kv: -kv[1]["total_ms"]):
                print(f"{k:20s} launches/step={v['launches'] / args.steps:6.1f} mean={v['mean_ms']:8.3f} ms "
                      f"algo={v['gbps']:8.1f} GB/s", file=sys.stderr)
        print(json.dumps(res))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
