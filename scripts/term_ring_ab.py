"""A/B of the term reverse's row kernels (grr_bwd_term_fused) on the training shapes, in one process:
level 1 = register-prefetch row kernel, level 2 = LDS-ring row kernel.  HIP-event time per launch,
two alternations per shape, algorithmic bytes as kernels.py counts them (x, g, v, w, gw read + write).

    python scripts/term_ring_ab.py [--iters 20] [--shapes msgf|c4|all]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {
    "msgf": [(16, 32, 3, 256, 256), (16, 32, 3, 128, 128)],
    "c4": [(32, 8, 6, 512, 512), (32, 8, 6, 256, 256), (32, 16, 6, 256, 256), (32, 16, 6, 128, 128),
           (32, 16, 12, 128, 128), (32, 16, 12, 64, 64), (32, 32, 12, 64, 64), (32, 32, 12, 32, 32)],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--shapes", default="all", choices=["msgf", "c4", "all"])
    ap.add_argument("--modes", default="0,1,2")
    args = ap.parse_args()
    import irdu_amd
    irdu_amd.load_native()
    from irdu_amd import kernels as K
    dev = torch.device("cuda", 0)
    shapes = SHAPES["msgf"] + SHAPES["c4"] if args.shapes == "all" else SHAPES[args.shapes]
    modes = [int(m) for m in args.modes.split(",")]
    for (b, g, f, h, w) in shapes:
        c = g * f
        torch.manual_seed(0)
        x = torch.randn(b, c, h, w, device=dev)
        gg = torch.randn(b, c, h, w, device=dev)
        taps = torch.randn(c, 5, device=dev) * 0.5
        sc = torch.rand(g, device=dev) + 0.5
        for mode in modes:
            wpl = 2 if mode == 1 else 4
            wt = torch.rand(b, g, wpl, h, w, device=dev)
            lg = torch.log(torch.full((g,), 0.05, device=dev)) if mode == 2 else None
            gw, gdot, gt = torch.zeros_like(wt), torch.zeros(g, device=dev), torch.zeros_like(taps)
            ggam = torch.zeros(g, device=dev) if mode == 2 else None
            nbytes = 4 * b * h * w * (3 * c + 3 * wpl * g)
            res = {1: [], 2: []}
            for _ in range(2):
                for level in (1, 2):
                    K.set_term_rows(level)
                    for _ in range(3):
                        K.bwd_term_fused(mode, x, gg, taps, wt, lg, sc, 0.5, gw, ggam, gdot, gt, g)
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(args.iters):
                        K.bwd_term_fused(mode, x, gg, taps, wt, lg, sc, 0.5, gw, ggam, gdot, gt, g)
                    e1.record()
                    torch.cuda.synchronize()
                    res[level].append(e0.elapsed_time(e1) / args.iters)
            r1, r2 = min(res[1]), min(res[2])
            print(f"B{b} G{g} F{f} {h}x{w} mode{mode}: reg {r1:.4f} ms ({nbytes / r1 / 1e6:.0f} GB/s)  "
                  f"ring {r2:.4f} ms ({nbytes / r2 / 1e6:.0f} GB/s)  speedup {r1 / r2:.3f}  "
                  f"[{' '.join(f'{v:.4f}' for v in res[1])} | {' '.join(f'{v:.4f}' for v in res[2])}]", flush=True)
            del wt, gw
    K.set_term_rows(True)


if __name__ == "__main__":
    main()
