"""The weight-gradient (grr_wgrad) and 1x1-GEMM (conv1x1) calls of one training step, by shape: launches,
mean time (HIP events around each call, the stream synchronised -- isolation timing, not the overlapped
step), TF/s on the algorithmic flops and the output-tile padding of the wgrad plan (128 x 96 tiles).

    python scripts/gemm_shapes.py [--model abstract] [--size 512] [--batch 32]
"""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="abstract", choices=["abstract", "msgf"])
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--batch", type=int, default=32)
    args = ap.parse_args()
    import irdu_amd
    from irdu_amd import kernels as K
    from irdu_amd import training as T
    from bench import synthetic_patches
    from bench_train import D_ARGS
    irdu_amd.load_native()
    dev = torch.device("cuda", 0)
    torch.manual_seed(2204)
    if args.model == "abstract":
        model = irdu_amd.AbtractMultiScaleGraphFilter(3, 3, n_cgd_iters=10, **D_ARGS)
    else:
        model = irdu_amd.MultiScaleGraphFilter(3, 3, ngraphs=32, n_cgd_iters=10)
    tr = T.Trainer(model, {"loss02_weight": 0.0, "loss03_weight": 0.0}, dev)
    clean, noisy = synthetic_patches(args.batch, seed=2204, h=args.size, w=args.size)
    noisy = noisy.permute(0, 2, 3, 1).contiguous().to(dev)
    clean = clean.permute(0, 2, 3, 1).contiguous().to(dev)
    tr.step(noisy, clean)
    torch.cuda.synchronize()

    stats = collections.defaultdict(list)
    orig = {"wgrad": K.wgrad, "conv1x1": K.conv1x1}

    def wrap(name):
        fn = orig[name]

        def run(*a, **kw):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            out = fn(*a, **kw)
            e1.record()
            torch.cuda.synchronize()
            if name == "wgrad":
                g, x = a[0], a[1]
                b, m = g.shape[:2]
                k = x.shape[1]
                p = g[0, 0].numel()
                key = (name, b, m, k, p)
                flops = 2.0 * b * m * k * p
            else:
                x, w = a[0], a[1]
                b, k = x.shape[:2]
                m = w.shape[0]
                p = x[0, 0].numel()
                key = (name, b, m, k, p)
                flops = 2.0 * b * m * k * p
            stats[key].append((e0.elapsed_time(e1), flops))
            return out
        return run

    K.wgrad = wrap("wgrad")
    K.conv1x1 = wrap("conv1x1")
    tr.step(noisy, clean)
    torch.cuda.synchronize()
    K.wgrad, K.conv1x1 = orig["wgrad"], orig["conv1x1"]

    def pad(m, k):   # the wgrad plan's padded output (best orientation, 128 x 96 tiles)
        f = lambda a, b: (-(-a // 128) * 128) * (-(-b // 96) * 96)  # noqa: E731
        return m * k / min(f(m, k), f(k, m))

    tot = collections.Counter()
    rows = []
    for key, v in stats.items():
        ms = sum(t for t, _ in v)
        fl = sum(f for _, f in v)
        tot[key[0]] += ms
        rows.append((ms, key, len(v), fl / ms / 1e9))
    for ms, key, n, tf in sorted(rows, reverse=True):
        name, b, m, k, p = key
        extra = f" tile-use {pad(m, k):.2f}" if name == "wgrad" else ""
        print(f"{name:8s} B={b:3d} M={m:5d} K={k:5d} P={p:7d}  x{n:3d}  {ms:8.3f} ms  {ms / n:7.3f} ms/call "
              f"{tf:7.1f} TF/s{extra}")
    print("totals (ms, isolated):", {k: round(v, 2) for k, v in tot.items()})


if __name__ == "__main__":
    main()
