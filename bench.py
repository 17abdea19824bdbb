"""Benchmark: 10-stage GGTV-GGLR image filter on sigma=25 noisy 256x256 RGB patches.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--no-cpu-baseline]

One "step" = one forward of the image-domain GGTV-GGLR filter (MultiScaleGraphFilter,
G=32 graphs x F=3, C=96, S=10 unrolled stages, v13 feature CNN; SURVEY.md §8(d) "P")
over one per-GPU batch of B=64 synthetic noisy patches already resident in HBM.
N>1: one process per GPU (under torchrun, or spawned by this script when started plainly with
--gpus N: benchlib.join_or_spawn), each rank filters its own batch (the path shards
by patch — no data-path collective; scaling "weak"); the timed region is bracketed by
barrier + synchronize on both sides and the max over ranks is reported.

Rank 0 prints ONE JSON line with the metric, the roofline of the dominant solver kernel
(grr_system_step2: two CG stages per launch; timed live with HIP events on its launch
stream) and the CPU baseline (the oracle, timed on this host's cores on a bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "MPix/sec + PSNR@σ=25, 10-stage GGTV-GGLR on 256×256 patches, 1/2/4/8 GPU"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BF16_MFMA_PEAK_TFLOPS = 16 * 157.3  # dense bf16 / fp16 MFMA rate (MI355X_MICROARCH.md: 1/16 of it is the f32 rate)
# LNB GEMM1 (head) runs each fp32 product as 3 fp16 MFMA products (exact 2-term split), GEMM2 (mix) as 6
# bf16 products (exact 3-term split): their ceilings in algorithmic fp32 flops are the rate / 3 and / 6
SPLIT_F16_PEAK_TFLOPS = BF16_MFMA_PEAK_TFLOPS / 3
SPLIT_BF16_PEAK_TFLOPS = BF16_MFMA_PEAK_TFLOPS / 6
G, CIN, STAGES, H, W, SIGMA = 32, 3, 10, 256, 256, 25.0


def synthetic_patches(n, seed, h=H, w=W):
    """Piecewise-smooth clean patches (uint8 grid) + RandomState(seed).normal(0,1)*sigma/255 noise
    cast to fp32, as environ/data/images_pair_restoration_dataset.py:105-108."""
    rs = np.random.RandomState(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    clean = np.empty((n, CIN, h, w), np.float32)
    for i in range(n):
        for c in range(CIN):
            fy, fx, ph = rs.uniform(0.5, 4.0), rs.uniform(0.5, 4.0), rs.uniform(0, 6.28)
            img = 0.5 + 0.3 * np.sin(2 * np.pi * fy * yy / h + ph) * np.cos(2 * np.pi * fx * xx / w)
            for _ in range(3):
                r0, c0 = rs.randint(0, h - h // 4), rs.randint(0, w - w // 4)
                img[r0:r0 + rs.randint(8, h // 3), c0:c0 + rs.randint(8, w // 3)] += rs.uniform(-0.3, 0.3)
            clean[i, c] = img
    clean = np.round(np.clip(clean, 0, 1) * 255.0) / 255.0
    noise = (rs.normal(0, 1, clean.shape) * (SIGMA / 255.0)).astype(np.float32)
    return torch.from_numpy(clean.astype(np.float32)), torch.from_numpy(clean.astype(np.float32) + noise)


TRAINED = os.path.join(ROOT, "tests", "golden", "msgf_trained_g32_s10.safetensors")


def build_model(device, seed=2204, trained=False):
    """Reference init (default conv init + the reference's solver init constants), except the
    final 1x1 projection, set to the per-colour mean over the G filtered copies so that the
    output is an image.  trained=True loads the weights fixture that
    scripts/train_psnr_fixture.py trained from this init (4,000 Adam steps on synthetic
    sigma-25 patches; safetensors, weights only), so PSNR is measured on a filter that denoises."""
    import irdu_amd
    torch.manual_seed(seed)
    m = irdu_amd.MultiScaleGraphFilter(CIN, CIN, ngraphs=G, n_cgd_iters=STAGES)
    with torch.no_grad():
        w = torch.zeros(CIN, G * CIN, 1, 1)
        for gi in range(G):
            for c in range(CIN):
                w[c, gi * CIN + c] = 1.0 / G
        m.linear_combination.weight.copy_(w)
    if trained:
        from safetensors.torch import load_file
        m.load_state_dict(load_file(TRAINED))
    return m.to(device).eval()


# the solver kernels at the bench shape: grr_system_step2 (two CG stages per launch, stages 1-8)
# and grr_system_step (W = 256 row waves: stages 0 and 9, or every stage with kernels.STEP2 = False)
STEP2_KERNEL = "graph_step2_kernel"
STEP_KERNEL = "graph_row_kernel<true, 1, 2, 4>"
TRAFFIC_FILES = {STEP2_KERNEL: "traffic_system_step2.json", STEP_KERNEL: "traffic_system_step.json"}


def _traffic(path, kernel_prefix, batch):
    """hbm_bytes_per_launch of a PMC summary (scripts/pmc_bench.sh: FETCH_SIZE / WRITE_SIZE passes
    over this bench at the same batch), or None when absent or measured on another workload --
    a per-launch byte count only compares with the algorithmic bytes of the same shape."""
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    if not d.get("kernel", "").startswith(kernel_prefix):
        return None
    if d.get("workload") != {"batch": batch, "size": 256}:
        return None
    return d.get("hbm_bytes_per_launch")


def load_traffic(kernel, batch):
    """Per-launch HBM bytes of the solver kernel `kernel` at this bench's batch (profiles/)."""
    return _traffic(os.path.join(ROOT, "profiles", TRAFFIC_FILES[kernel]), kernel, batch)


def load_traffic_file(name, kernel_prefix, batch):
    """Per-launch HBM bytes (mean over the bench's launches of that kernel): the newest round's summary
    under profiles/ of this workload."""
    for rnd in ("r06", "r05", "r04", "r03"):
        t = _traffic(os.path.join(ROOT, "profiles", rnd, name), kernel_prefix, batch)
        if t is not None:
            return t
    return None


def host_cpus():
    """(os.cpu_count(), CPUs this process may use: affinity mask and cgroup CPU quota)."""
    n = os.cpu_count() or 1
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else n
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            usable = min(usable, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n, usable


def cpu_model():
    cpu = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return cpu


def cpu_baseline(model_cpu_state, n_img=1, runs=3):
    """the oracle (the reference's op sequence in PyTorch-CPU fp32; timed against
    the reference itself in the build container at a ratio of 1.01-1.05, profiles/r02/
    calibrate_oracle_256.json) on a bounded sample of the workload -- n_img 256x256 patches, S = 10,
    G = 32 -- with torch.set_num_threads(os.cpu_count()) (capped at the CPUs the process may
    actually run on: affinity mask / cgroup quota, both printed), one warm-up, median of `runs`."""
    import statistics
    from oracle import graph_oracle as O
    n_cpu, usable = host_cpus()
    threads = min(n_cpu, usable)
    torch.set_num_threads(threads)
    clean, noisy = synthetic_patches(n_img, seed=99)
    times = []
    with torch.no_grad():
        O.multiscale_graph_filter(noisy[:, :, :64, :64], model_cpu_state, G)   # warm-up (allocator, pool)
        for _ in range(runs):
            t0 = time.perf_counter()
            ref = O.multiscale_graph_filter(noisy, model_cpu_state, G)
            times.append(time.perf_counter() - t0)
    dt = statistics.median(times)
    mpix = n_img * H * W / dt / 1e6
    return {"value": mpix, "unit": "MPix/s", "cores": threads, "kind": "port",
            "sample": f"{n_img} patch(es) {H}x{W} RGB sigma=25, S={STAGES}, G={G}: median of {runs} runs "
                      f"{dt:.2f} s (runs {', '.join(f'{t:.2f}' for t in times)}) on {cpu_model()}",
            "runs": runs, "median_s": round(dt, 3), "os_cpu_count": n_cpu, "usable_cpus": usable,
            "restatement_over_reference": "1.01-1.05 (build container, profiles/r02/calibrate_oracle_256.json)"}, \
        clean, noisy, ref


D_CFG = dict(dims=[48, 96, 192, 384], hidden_dims=[96, 192, 384, 768], nsubnets=[1, 1, 1, 1],
             ngraphs=[8, 16, 16, 32], num_blocks=[4, 6, 6, 8], num_blocks_out=4)


def bench_abstract(dev, b, steps=3):
    """SURVEY.md §8(d) 'D': the drop-in v1.0 AbtractMultiScaleGraphFilter (trained dims of
    README.ipynb:74-84) with S = 10 in all four filter blocks: end-to-end forward and the
    filtering() part alone, on b synthetic 256x256 patches (rank 0 only, after the main timing)."""
    import irdu_amd
    torch.manual_seed(2204)
    m = irdu_amd.AbtractMultiScaleGraphFilter(3, 3, n_cgd_iters=STAGES, **D_CFG).to(dev).eval()
    _, noisy = synthetic_patches(b, seed=7)
    noisy = noisy.to(dev)
    with torch.no_grad():
        for _ in range(2):
            m(noisy)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            m(noisy)
        torch.cuda.synchronize(dev)
        t_full = (time.perf_counter() - t0) / steps
        coefs = m.encode(noisy)
        m.filtering(coefs)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            m.filtering(coefs)
        torch.cuda.synchronize(dev)
        t_filt = (time.perf_counter() - t0) / steps
    px = b * H * W
    return {"workload": f"AbtractMultiScaleGraphFilter v1.0 dims {D_CFG['dims']} ngraphs {D_CFG['ngraphs']} "
                        f"blocks {D_CFG['num_blocks']}, S={STAGES} in all 4 filter blocks, {H}x{W} RGB",
            "per_gpu_batch": b, "mpix_per_s": round(px / t_full / 1e6, 3), "ms_per_step": round(t_full * 1e3, 2),
            "filtering_mpix_per_s": round(px / t_filt / 1e6, 3), "filtering_ms": round(t_filt * 1e3, 2),
            "note": "encoder/decoder plain convs on stock PyTorch-ROCm; every LocalNonLinearBlock and filter "
                    "block on HIP"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 40 steps ~ 1.7 s of GPU time: long enough for an external utilisation sampler to see the run
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64, help="patches per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the secondary workload (v1.0 AbtractMultiScaleGraphFilter, SURVEY.md §8d 'D')")
    ap.add_argument("--breakdown", action="store_true", help="print the per-kernel table to stderr")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check: every rank prints its rank / world and exits (no HIP)")
    args = ap.parse_args()

    # --gpus N: one process per GPU.  Under torchrun the ranks exist already (WORLD_SIZE must
    # equal N); started plainly, this process spawns the N ranks and exits with their status
    import benchlib
    world, rank, local = benchlib.join_or_spawn(args.gpus, dry_run=args.dry_run)
    if args.dry_run:
        benchlib.dry_run_report(world, rank, local)
        return
    dev = benchlib.init(world, local)
    ranks = benchlib.check_ranks(world, dev)     # every rank in the group, over the data backend

    import irdu_amd
    from irdu_amd import kernels as K
    irdu_amd.load_native()
    model = build_model(dev, trained=os.path.exists(TRAINED))
    b = args.batch
    # each rank its own shard of patches (seed by rank): resident in HBM before timing
    _, noisy = synthetic_patches(b, seed=2204 + rank)
    noisy = noisy.to(dev)

    def barrier():
        benchlib.barrier(world, dev)

    with torch.no_grad():
        for _ in range(args.warmup):
            out = model(noisy)
        # headline: a clean timed loop (no per-launch instrumentation)
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = model(noisy)
        barrier()
        dt = time.perf_counter() - t0
        # then the same steps again with HIP events around every launch (per-kernel breakdown and
        # the roofline's kernel time); this loop's wall time is not the headline.  It runs on one
        # stream (no feature side stream), so each kernel's time is its own and not shared with a
        # concurrent kernel
        from irdu_amd import graph_filter as GF
        saved = GF.FEATURE_STREAMS
        GF.FEATURE_STREAMS = False
        timer = K.LaunchTimer()
        timer.split_lnb = True      # the feature CNN's head and mix kernels timed apart
        K.set_timer(timer)
        for _ in range(max(1, min(args.steps, 5))):
            out = model(noisy)
        K.set_timer(None)
        GF.FEATURE_STREAMS = saved
        n_inst = max(1, min(args.steps, 5))
    kern = timer.summary()
    rank_dts = [r[0] for r in benchlib.gather_floats([dt], world, dev)]
    dt = benchlib.max_over_ranks(dt, world, dev)
    if rank != 0:
        benchlib.finish(world)
        return

    px_total = world * b * H * W * args.steps
    value = px_total / dt / 1e6
    # the dominant solver kernel: the two-stage launch where the filter uses it
    kind, kname = ("system_step2", STEP2_KERNEL) if "system_step2" in kern else ("system_step", STEP_KERNEL)
    step = kern[kind]
    achieved = step["gbps"]
    traffic = load_traffic(kname, b)
    roofline = {"bound": "hbm", "kernel": f"grr_{kind} ({kname})",
                "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                "bytes_per_launch": step["bytes_per_launch"], "mean_launch_ms": round(step["mean_ms"], 4),
                "launches": step["launches"]}
    if kind == "system_step2":
        roofline["stages_per_launch"] = 2
        roofline["ms_per_stage"] = round(step["mean_ms"] / 2, 4)
    # context for frac: a float4 streaming copy's rate on this GPU (read + write bytes / time),
    # i.e. what a pure streaming kernel reaches here; measured after the timed region
    src = torch.empty(1 << 30, dtype=torch.float32, device=dev)
    dst = torch.empty_like(src)
    K.stream_copy(src, dst)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        K.stream_copy(src, dst)
    e1.record()
    torch.cuda.synchronize(dev)
    copy_gbps = 10 * 2 * src.numel() * 4 / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del src, dst
    roofline["copy_gbps"] = round(copy_gbps, 1)
    roofline["frac_of_copy"] = round(achieved / copy_gbps, 4)
    res = {"metric": METRIC, "value": round(value, 3), "unit": "MPix/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
           "config": {"workload": "MultiScaleGraphFilter (image-domain GGTV-GGLR, v13 feature CNN) "
                                  f"G={G} F={CIN} C={G * CIN}, S={STAGES} stages, {H}x{W} RGB sigma=25, "
                                  + ("weights: trained fixture" if os.path.exists(TRAINED) else
                                     "reference-init weights, output 1x1 = per-colour graph mean"),
                      "global_batch": world * b, "per_gpu_batch": b, "image": f"{H}x{W}x{CIN}",
                      "parallelism": f"batch-sharded x{world}, no collective in the data path"},
           "roofline": roofline}
    if world > 1:
        res.update(ranks)
        res["ranks"] = {"backend": ranks["backend"], "visible_gpus": torch.cuda.device_count(),
                        "ms_per_step_per_rank": [round(d / args.steps * 1e3, 3) for d in rank_dts]}
    if "lnb_head" in kern:   # the feature CNN: head (LN + W1 + depthwise + gate) and mix (W2 + skip) apart
        hd, mx = kern["lnb_head"], kern["lnb_mix"]
        res["roofline_secondary"] = {
            "lnb_head": {
                "bound": "mfma", "kernel": "lnb_head16_kernel (+ lnb_w1_pack16_kernel)",
                "achieved": round(hd["tflops"], 2), "peak": round(SPLIT_F16_PEAK_TFLOPS, 1), "unit": "TFLOP/s",
                "frac": round(hd["tflops"] / SPLIT_F16_PEAK_TFLOPS, 4), "flops_per_launch": hd["flops_per_launch"],
                "mean_launch_ms": round(hd["mean_ms"], 4), "launches": hd["launches"],
                "traffic": load_traffic_file("traffic_lnb_head16.json", "lnb_head16_kernel", b),
                "note": "algorithmic fp32 flops (kernels.lnb_head_flops: LN, W1, depthwise, gate) / HIP-event time, "
                        "against the dense fp16 MFMA rate / 3 (each W1 product = 3 fp16 products of exact 2-term "
                        "splits); the depthwise + gate part is VALU work"},
            "lnb_mix": {
                "bound": "hbm", "kernel": "lnb_mix_kernel (+ lnb_w2_pack_kernel)",
                "achieved": round(mx["gbps"], 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(mx["gbps"] / HBM_PEAK_GBPS, 4), "bytes_per_launch": mx["bytes_per_launch"],
                "mean_launch_ms": round(mx["mean_ms"], 4), "launches": mx["launches"],
                "mfma_tflops": round(mx["tflops"], 2), "mfma_peak": round(SPLIT_BF16_PEAK_TFLOPS, 1),
                "traffic": load_traffic_file("traffic_lnb_mix.json", "lnb_mix_kernel", b),
                "note": "algorithmic bytes (g + skip operand + out) / HIP-event time; W2 on 6 bf16 products"}}
    if "lnb_fused" in kern:   # the C = 96 blocks as one fused pass (lnb_fused16_kernel)
        fu = kern["lnb_fused"]
        res.setdefault("roofline_secondary", {})["lnb_fused"] = {
            "bound": "mfma", "kernel": "lnb_fused16_kernel (+ lnb_fused_pack_kernel)",
            "achieved": round(fu["tflops"], 2), "peak": round(SPLIT_F16_PEAK_TFLOPS, 1), "unit": "TFLOP/s",
            "frac": round(fu["tflops"] / SPLIT_F16_PEAK_TFLOPS, 4), "flops_per_launch": fu["flops_per_launch"],
            "mean_launch_ms": round(fu["mean_ms"], 4), "launches": fu["launches"],
            "hbm_gbps": round(fu["gbps"], 1), "bytes_per_launch": fu["bytes_per_launch"],
            "traffic": load_traffic_file("traffic_lnb_fused.json", "lnb_fused16_kernel", b),
            "note": "algorithmic fp32 flops (LN, W1, depthwise, gate, W2, skip) / HIP-event time against the dense "
                    "fp16 rate / 3 (both GEMMs on exact fp16 two-term splits, three products each); bytes: x in, out "
                    "written (compulsory); the gated activation stays on chip"}
    if "lnb_rep_fused" in kern:   # the first block, on the replicated RGB input: one fused pass
        rp = kern["lnb_rep_fused"]
        res.setdefault("roofline_secondary", {})["lnb_rep_fused"] = {
            "bound": "mfma", "kernel": "lnb_rep_kernel (+ lnb_rep_pack_kernel)",
            "achieved": round(rp["tflops"], 2), "peak": round(SPLIT_F16_PEAK_TFLOPS, 1), "unit": "TFLOP/s",
            "frac": round(rp["tflops"] / SPLIT_F16_PEAK_TFLOPS, 4), "flops_per_launch": rp["flops_per_launch"],
            "mean_launch_ms": round(rp["mean_ms"], 4), "launches": rp["launches"],
            "hbm_gbps": round(rp["gbps"], 1), "bytes_per_launch": rp["bytes_per_launch"],
            "traffic": load_traffic_file("traffic_lnb_rep.json", "lnb_rep_kernel", b),
            "note": "algorithmic fp32 flops (LN, W1, depthwise, gate, W2, skip) / HIP-event time against the "
                    "dense fp16 rate / 3 (both GEMMs on exact fp16 two-term splits; the depthwise folded into "
                    "GEMM1 as a 27-deep im2col operand); bytes: src in, out written"}
    if "system_first_pair" in kern:   # stage 0 + prox rhs B + stage 1 in one pass
        fp = kern["system_first_pair"]
        res.setdefault("roofline_secondary", {})["system_first_pair"] = {
            "bound": "hbm", "kernel": "graph_step2_kernel<false, false, true> (grr_system_first_pair)",
            "achieved": round(fp["gbps"], 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(fp["gbps"] / HBM_PEAK_GBPS, 4), "bytes_per_launch": fp["bytes_per_launch"],
            "mean_launch_ms": round(fp["mean_ms"], 4), "launches": fp["launches"],
            "traffic": load_traffic_file("traffic_system_first_pair.json", "graph_step2_kernel", b),
            "note": "algorithmic bytes (kernels.first_pair_bytes: b_A, D b_A, y, three full- and three half-level "
                    "weight planes sets read once; b_B, x_2, u_2, D x_2 written) / HIP-event time"}
    if "feature_edges" in kern:   # a level's feature 1x1 + both graph modules' edge weights in one pass
        fe = kern["feature_edges"]
        res.setdefault("roofline_secondary", {})["feature_edges"] = {
            "bound": "hbm", "kernel": "feat_edge_kernel (grr_feature_edges)",
            "achieved": round(fe["gbps"], 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(fe["gbps"] / HBM_PEAK_GBPS, 4), "bytes_per_launch": fe["bytes_per_launch"],
            "mean_launch_ms": round(fe["mean_ms"], 4), "launches": fe["launches"],
            "traffic": load_traffic_file("traffic_feature_edges.json", "feat_edge_kernel", b),
            "note": "algorithmic bytes (kernels.feature_edges: 4 (C + 10 G) per pixel -- the LocalNonLinearBlock output "
                    "in, the GTV raw and pair weights and the GLR raw weights out; the 2C features never reach HBM) / "
                    "HIP-event time"}
    kernels_ms = {k: round(v["total_ms"] / n_inst, 3) for k, v in kern.items()}
    res["kernel_ms_per_step"] = kernels_ms
    if args.breakdown:
        for k, v in sorted(kern.items(), key=lambda kv: -kv[1]["total_ms"]):
            print(f"{k:18s} launches/step={v['launches'] / n_inst:5.1f} mean={v['mean_ms']:8.3f} ms "
                  f"algo={v['gbps']:8.1f} GB/s", file=sys.stderr)
    # the secondary workload and the CPU baseline (+ PSNR parity) belong to the N = 1 line;
    # the N > 1 lines of the scaling run carry throughput and the roofline only
    if not args.no_secondary and world == 1:
        res["secondary_workload"] = bench_abstract(dev, min(b, 16))
    if not args.no_cpu_baseline and world == 1:
        from oracle import graph_oracle as O
        state = {k: v.detach().cpu() for k, v in model.state_dict().items()}
        cb, clean, cnoisy, ref = cpu_baseline(state)
        with torch.no_grad():
            got = model(cnoisy.to(dev)).cpu()
        rel = float((got.double() - ref.double()).abs().max() / ref.double().abs().max())
        p_gpu, p_cpu = O.psnr_ubyte(got, clean), O.psnr_ubyte(ref, clean)
        res["cpu_baseline"] = {k: (round(v, 5) if isinstance(v, float) else v) for k, v in cb.items()}
        res["psnr"] = {"gpu_db": round(p_gpu, 4), "oracle_db": round(p_cpu, 4), "delta_db": round(abs(p_gpu - p_cpu), 5),
                       "noisy_input_db": round(O.psnr_ubyte(cnoisy, clean), 4), "rel_err_vs_oracle": rel,
                       "weights": ("tests/golden/msgf_trained_g32_s10.safetensors (trained here: no reference "
                                   "checkpoint exists)") if os.path.exists(TRAINED) else "reference init"}
        res["speedup_vs_cpu"] = round(value / world / cb["value"], 1)
    print(json.dumps(res), flush=True)
    benchlib.finish(world)


if __name__ == "__main__":
    main()
