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


HBM_PEAK_GBPS = 8000.0


def load_traffic(kind, model, batch, size):
    """Per-launch HBM bytes (PMC, scripts/pmc_train.sh) of the reverse kernel kind at this workload,
    or None when no summary of that exact shape is committed under profiles/."""
    for rnd, name in (("r04", f"traffic_{kind}_{model}_b{batch}_s{size}.json"), ("r04", f"traffic_{kind}_{model}.json"),
                      ("r03", f"traffic_{kind}_{model}.json")):   # the newest summary of this exact workload
        path = os.path.join(ROOT, "profiles", rnd, name)
        if not os.path.exists(path):
            continue
        with open(path) as f:
            d = json.load(f)
        shape = d.get("workload", {})
        if shape and (shape.get("batch"), shape.get("size")) != (batch, size):
            continue
        return d.get("hbm_bytes_per_launch")
    return None


def reverse_roofline(kern, model, batch, size):
    """Roofline of the dominant reverse-sweep kernel kind: algorithmic bytes per launch
    (kernels.py byte model of each reverse pass) / its mean HIP-event launch time; traffic = the PMC
    bytes per launch of the same kind (profiles/r03/traffic_<kind>_<model>.json)."""
    cands = {k: v for k, v in kern.items() if k.startswith("bwd") and v["bytes_per_launch"] > 0}
    if not cands:
        return None
    k, v = max(cands.items(), key=lambda kv: kv[1]["total_ms"])
    return {"bound": "hbm", "kernel": k, "achieved": round(v["gbps"], 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(v["gbps"] / HBM_PEAK_GBPS, 4), "traffic": load_traffic(k, model, batch, size),
            "bytes_per_launch": v["bytes_per_launch"], "mean_launch_ms": round(v["mean_ms"], 4),
            "launches": v["launches"]}


BF16_MFMA_PEAK_TFLOPS = 2500.0   # MI355X_MICROARCH.md: dense bf16 / fp16 MFMA
SPLIT_BF16_PEAK_TFLOPS = BF16_MFMA_PEAK_TFLOPS / 6   # six bf16 products per fp32-accurate product


def secondary_rooflines(kern):
    """Rooflines of the training step's other large kernel families: the split-bf16 GEMMs (conv1x1: every
    1x1 conv / LNB GEMM data path; wgrad: the weight gradients) against the dense bf16 MFMA rate / 6 (each
    fp32-accurate product = six bf16 products of exact three-term splits), and the LNB gate + depthwise
    reverse (a streaming row kernel) against HBM; algorithmic flops / bytes over HIP-event time."""
    out = {}
    for kind, label in (("conv1x1", "gemm_x3_kernel / gemm_x3k_kernel (1x1 convs, LNB GEMMs, 2x2 data grads)"),
                        ("wgrad", "wgrad_kernel + its fixed-order chunk reduction (weight gradients)")):
        v = kern.get(kind)
        if v and v["flops_per_launch"] > 0:
            out[kind] = {"bound": "mfma", "kernel": label, "achieved": round(v["tflops"], 2),
                         "peak": round(SPLIT_BF16_PEAK_TFLOPS, 1), "unit": "TFLOP/s",
                         "frac": round(v["tflops"] / SPLIT_BF16_PEAK_TFLOPS, 4),
                         "flops_per_launch": v["flops_per_launch"], "mean_launch_ms": round(v["mean_ms"], 4),
                         "launches": v["launches"], "hbm_gbps": round(v["gbps"], 1)}
    for kind in ("lnb_gate_dw3_bwd", "lnb_norm_bwd", "bwd_cg_glue"):
        v = kern.get(kind)
        if v and v["bytes_per_launch"] > 0:
            out[kind] = {"bound": "hbm", "achieved": round(v["gbps"], 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(v["gbps"] / HBM_PEAK_GBPS, 4), "bytes_per_launch": v["bytes_per_launch"],
                         "mean_launch_ms": round(v["mean_ms"], 4), "launches": v["launches"]}
    return out


def cpu_baseline(model, model_kind, size, runs=3):
    """The oracle's differentiable restatement of the same model (PyTorch-CPU fp32, the
    reference's op sequence) for one optimisation step -- forward, L1 loss, autograd reverse,
    Adam -- on one size x size patch; threads = the CPUs this process may use; median of runs."""
    import statistics
    from bench import cpu_model, host_cpus, synthetic_patches
    from oracle import graph_oracle as O
    n_cpu, usable = host_cpus()
    threads = min(n_cpu, usable)
    torch.set_num_threads(threads)
    names = {k for k, _ in model.named_parameters()}
    state = {k: v.detach().cpu().clone().requires_grad_(k in names) for k, v in model.state_dict().items()}
    params = [v for v in state.values() if v.requires_grad]
    opt = torch.optim.Adam(params, lr=4e-4, eps=1e-8)
    clean, noisy = synthetic_patches(1, seed=99, h=size, w=size)

    def fwd(x):
        if model_kind == "msgf":
            return O.multiscale_graph_filter(x, state, 32)
        return O.abstract_forward(x, state, D_ARGS["ngraphs"], D_ARGS["num_blocks"], D_ARGS["num_blocks_out"],
                                  D_ARGS["nsubnets"])

    def step(x, c):
        opt.zero_grad(set_to_none=True)
        loss = torch.nn.functional.l1_loss(fwd(x), c)
        loss.backward()
        opt.step()

    step(noisy[..., :32, :32], clean[..., :32, :32])   # warm-up
    times = []
    for _ in range(runs):
        t0 = time.perf_counter()
        step(noisy, clean)
        times.append(time.perf_counter() - t0)
    dt = statistics.median(times)
    return {"value": round(size * size / dt / 1e6, 6), "unit": "MPix/s", "cores": threads, "kind": "port",
            "sample": f"1 patch {size}x{size} RGB sigma=25, forward + L1 + autograd reverse + Adam: median of "
                      f"{runs} steps {dt:.2f} s (runs {', '.join(f'{t:.2f}' for t in times)}) on {cpu_model()}",
            "os_cpu_count": n_cpu, "usable_cpus": usable}


def main():
    # process-wide MIOpen setting of the training entry points, before any convolution (training.py)
    os.environ.setdefault("MIOPEN_DEBUG_DISABLE_FIND_DB", "1")
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", choices=["abstract", "msgf"], default="abstract")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--batch", type=int, default=8, help="patches per GPU")
    ap.add_argument("--stages", type=int, default=10)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--aux-losses", action="store_true", help="add the enc-dec / latent-perturbation losses")
    ap.add_argument("--breakdown", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-size", type=int, default=None,
                    help="CPU-baseline patch side (default: --size for msgf, 128 for the v1.0 model)")
    ap.add_argument("--fused-fts", type=str, default=None,
                    help="comma list of F that use the one-pass term reverses (default: all instances)")
    ap.add_argument("--keep-gate", type=int, choices=[0, 1], default=1,
                    help="LNB forward keeps the gated activation for the reverse (solver_grad.KEEP_GATE; A/B runs)")
    ap.add_argument("--term-acc", type=int, choices=[0, 1], default=1,
                    help="x-gradient pass inside the term reverse (solver_grad.TERM_ACC; A/B runs)")
    ap.add_argument("--unpool-glue", type=int, choices=[0, 1], default=1,
                    help="half level's U folded into the next glue pass (solver_grad.UNPOOL_GLUE; A/B runs)")
    ap.add_argument("--padj-glue", type=int, choices=[0, 1], default=1,
                    help="full level's x-gradient sweep folded into the next glue pass (solver_grad.PADJ_GLUE; A/B)")
    ap.add_argument("--ln-skip", type=int, choices=[0, 1], default=1,
                    help="LNB skip term inside the norm's reverse pass (solver_grad.LN_SKIP_FUSED; A/B runs)")
    ap.add_argument("--watchdog", type=float, default=0.0,
                    help="dump every thread's Python stack to stderr each N seconds (hang diagnosis)")
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one process per GPU; spawned when not under torchrun)")
    ap.add_argument("--dry-run", action="store_true", help="launcher check: ranks report and exit (no HIP)")
    ap.add_argument("--conv-benchmark", action="store_true",
                    help="torch.backends.cudnn.benchmark: MIOpen Find for the stock convolutions")
    args = ap.parse_args()
    if args.conv_benchmark:
        torch.backends.cudnn.benchmark = True

    if args.watchdog > 0:
        import faulthandler
        faulthandler.dump_traceback_later(args.watchdog, repeat=True, file=sys.stderr)
    import benchlib
    world, rank, local = benchlib.join_or_spawn(args.gpus, dry_run=args.dry_run)
    if args.dry_run:
        benchlib.dry_run_report(world, rank, local)
        return
    dev = benchlib.init(world, local)
    ranks = benchlib.check_ranks(world, dev)     # every rank in the group, over the data backend

    import irdu_amd
    from irdu_amd import kernels as K
    from irdu_amd import training as T
    from bench import synthetic_patches
    irdu_amd.load_native()
    if args.fused_fts is not None:
        K.FUSED_TERM_FTS = tuple(int(v) for v in args.fused_fts.split(",") if v)
    from irdu_amd import solver_grad as SGK
    SGK.KEEP_GATE = bool(args.keep_gate)
    SGK.TERM_ACC = bool(args.term_acc)
    SGK.UNPOOL_GLUE = bool(args.unpool_glue)
    SGK.PADJ_GLUE = bool(args.padj_glue)
    SGK.LN_SKIP_FUSED = bool(args.ln_skip)
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
        benchlib.barrier(world, dev)

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
    dt = benchlib.max_over_ranks(dt, world, dev)
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
        if world > 1:
            res.update(ranks)
        res["roofline"] = reverse_roofline(kern, args.model, args.batch, args.size)
        res["roofline_secondary"] = secondary_rooflines(kern)
        if not args.no_cpu_baseline and world == 1:
            cb = cpu_baseline(model, args.model, args.cpu_size or (args.size if args.model == "msgf" else 128))
            res["cpu_baseline"] = cb
            res["speedup_vs_cpu"] = round(res["value"] / cb["value"], 1)
        if args.breakdown:
            for k, v in sorted(kern.items(), key=lambda kv: -kv[1]["total_ms"]):
                print(f"{k:20s} launches/step={v['launches'] / args.steps:6.1f} mean={v['mean_ms']:8.3f} ms "
                      f"algo={v['gbps']:8.1f} GB/s", file=sys.stderr)
        print(json.dumps(res), flush=True)
    benchlib.finish(world)
    if args.watchdog > 0:
        import faulthandler
        faulthandler.cancel_dump_traceback_later()


if __name__ == "__main__":
    main()
