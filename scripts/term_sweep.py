"""Per-shape timing of the training reverse's operator-term pass (grr_bwd_term_fused / _acc) at the
shapes one model's training step launches it with (C4: the v1.0 model at 512^2 x 32), for each term
row kernel level.  HIP events around N launches; GB/s from the same algorithmic bytes as bench_train.

    python scripts/term_sweep.py [--batch 32] [--size 512] [--iters 10] [--rows 1,2]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import irdu_amd  # noqa: E402
from irdu_amd import kernels as K  # noqa: E402

# v1.0 (AbtractMultiScaleGraphFilter): dims, graphs per encoder level; each level solves at full and half
DIMS, GRAPHS = [48, 96, 192, 384], [8, 16, 16, 32]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rows", default="1,2")
    ap.add_argument("--modes", default="0,1,2")
    ap.add_argument("--levels", default="", help="comma list of shapes to run (L0f,L0h,...; default all)")
    ap.add_argument("--tail", default="1", help="comma list of grr_bwd_set_term_tail settings (0,1)")
    args = ap.parse_args()
    irdu_amd.load_native()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    total = {}
    for lvl, (c, g) in enumerate(zip(DIMS, GRAPHS)):
        for half in (0, 1):
            s = args.size >> (lvl + half)
            if args.levels and f"L{lvl}{'h' if half else 'f'}" not in args.levels.split(","):
                continue
            b = args.batch
            x = torch.randn(b, c, s, s, device=dev)
            gg = torch.randn_like(x)
            taps = torch.randn(c, 5, device=dev) * 0.5
            sc = torch.rand(g, device=dev) + 0.5
            for mode in map(int, args.modes.split(",")):
                wt = torch.rand(b, g, 2 if mode == 1 else 4, s, s, device=dev)
                lg = torch.log(torch.full((g,), 0.05, device=dev)) if mode == 2 else None
                gw, gdot, gt = torch.zeros_like(wt), torch.zeros(g, device=dev), torch.zeros_like(taps)
                ggam = torch.zeros(g, device=dev) if mode == 2 else None
                gx = torch.zeros_like(x)
                nbytes = 4 * (3 * x.numel() + 3 * wt.numel())
                line = f"L{lvl}{'h' if half else 'f'} C={c:3d} G={g:2d} F={c // g:2d} {s:3d}^2 mode {mode}:"
                for rows, tail in [(r, t) for r in map(int, args.rows.split(",")) for t in map(int, args.tail.split(","))]:
                    K.set_term_rows(rows)
                    K.set_term_tail(bool(tail))
                    acc = K.term_acc_ok(mode, x, g, gg, wt)
                    if acc:
                        fn = lambda: K.bwd_term_fused_acc(mode, x, gg, taps, wt, lg, sc, 0.5, gx, gw, ggam, gdot, gt, g)  # noqa: E731
                    else:
                        fn = lambda: K.bwd_term_fused(mode, x, gg, taps, wt, lg, sc, 0.5, gw, ggam, gdot, gt, g)  # noqa: E731
                    with torch.no_grad():
                        for _ in range(2):
                            fn()
                        torch.cuda.synchronize()
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        for _ in range(args.iters):
                            fn()
                        e1.record()
                        torch.cuda.synchronize()
                    ms = e0.elapsed_time(e1) / args.iters
                    key = (rows, tail)
                    total[key] = total.get(key, 0.0) + ms
                    line += f"  rows{rows}{'+acc' if acc else ''} t{tail} {ms:7.3f} ms {nbytes / ms / 1e6:7.1f} GB/s"
                print(line, flush=True)
                del wt, gw
    K.set_term_rows(True)
    K.set_term_tail(True)
    print("sum of one launch per (shape, mode):", {f"rows{k[0]} t{k[1]}": round(v, 3) for k, v in total.items()})


if __name__ == "__main__":
    main()
