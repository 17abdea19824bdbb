"""Wide-image benchmark: the bench's image filter on images wider than 256 columns.

    python bench_wide.py [--size 512x512] [--batch 16] [--steps 5] [--warmup 2] [--compare] [--compare-step2]

W > 256 runs the CG stage pairs as two-stage passes in column strips (grr_system_step2: 256-lane
windows, 224 owned columns, 16 halo columns per side) and the remaining graph operators as V = 4 row
waves in column strips (248 output columns, 4 halo columns per side, graph_row_kernel);
--compare-step2 also times one launch per stage (kernels.STEP2_STRIPS = False), --compare the 64-column strip
kernels (grr_set_kernel_variant(1), graph_op_kernel) on the same batch.  Not the headline metric (bench.py
is); prints one JSON line per variant with MPix/s and the per-kernel-kind time.
Configs: 512x512 (config C4's image size), 336x496 (the BSD68 eval crops' landscape size).
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
    ap.add_argument("--size", default="512x512", help="HxW")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--compare", action="store_true", help="also time the 64-column strip kernels")
    ap.add_argument("--compare-step2", action="store_true", help="also time one launch per CG stage")
    args = ap.parse_args()
    h, w = (int(v) for v in args.size.lower().split("x"))
    import irdu_amd
    from irdu_amd import kernels as K
    from bench import TRAINED, build_model, synthetic_patches
    irdu_amd.load_native()
    dev = torch.device("cuda", 0)
    model = build_model(dev, trained=os.path.exists(TRAINED))
    _, noisy = synthetic_patches(args.batch, seed=11, h=h, w=w)
    noisy = noisy.to(dev)
    outs = {}
    variants = ["auto"] + (["strips"] if args.compare else []) + (["per_stage"] if args.compare_step2 else [])
    for variant in variants:
        K.set_kernel_variant("auto" if variant == "per_stage" else variant)
        K.STEP2_STRIPS = variant != "per_stage"
        with torch.no_grad():
            for _ in range(args.warmup):
                model(noisy)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(args.steps):
                out = model(noisy)
            torch.cuda.synchronize(dev)
            dt = (time.perf_counter() - t0) / args.steps
            timer = K.LaunchTimer()
            K.set_timer(timer)
            model(noisy)
            K.set_timer(None)
        outs[variant] = out
        kern = timer.summary()
        row = {"metric": "wide-image MPix/s (forward, 1 GPU)", "value": round(args.batch * h * w / dt / 1e6, 3),
               "unit": "MPix/s", "ms_per_step": round(dt * 1e3, 2), "image": f"{h}x{w}x3", "batch": args.batch,
               "graph_kernels": {"auto": "stage pairs in two-stage strip passes, row waves in 248-column strips",
                                 "strips": "64-column strips (graph_op_kernel)",
                                 "per_stage": "one launch per CG stage, row waves in 248-column strips"}[variant],
               "two_stage_passes": bool(K.STEP2 and K.STEP2_STRIPS and w > 256 and w % 8 == 0),
               "kernel_ms": {k: round(v["total_ms"], 3) for k, v in kern.items()},
               "kernel_gbps": {k: round(v["gbps"], 1) for k, v in kern.items() if v["gbps"] > 0}}
        print(json.dumps(row), flush=True)
    K.set_kernel_variant("auto")
    K.STEP2_STRIPS = True
    if args.compare_step2:
        a, b = outs["auto"].double(), outs["per_stage"].double()
        print(json.dumps({"max_rel_diff_step2_vs_per_stage": float((a - b).abs().max() / b.abs().max())}))
    if args.compare:
        a, b = outs["auto"].double(), outs["strips"].double()
        print(json.dumps({"max_rel_diff_auto_vs_strips": float((a - b).abs().max() / b.abs().max())}))


if __name__ == "__main__":
    main()
