"""Micro-benchmark of single HIP kernels at the bench shape (P: B=64, G=32, F=3, 256x256).

    python scripts/micro.py [--kernel step|step2|half|lnb|lnb_rep|conv1x1|term|edge] [--iters N] [--batch B]

Used under rocprofv3 (kernel trace / PMC passes) to profile one kernel in isolation.
Prints mean milliseconds per launch and algorithmic GB/s from HIP events.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import irdu_amd  # noqa: E402
from irdu_amd import kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="step")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--variant", default="auto", choices=["auto", "strips", "independent"])
    ap.add_argument("--graphs", type=int, default=32)
    ap.add_argument("--fts", type=int, default=3)
    ap.add_argument("--split", action="store_true", help="LNB: time the head and the mix apart")
    ap.add_argument("--lnb-fused", type=int, default=1, choices=[0, 1],
                    help="LNB, C <= 96: 1 the fused pass, 0 the head + mix kernels (grr_lnb_set_fused)")
    ap.add_argument("--hid", type=int, default=256, help="LNB hidden width")
    ap.add_argument("--cin", type=int, default=192, help="conv_mk: input channels")
    ap.add_argument("--cout", type=int, default=48, help="conv_mk: output channels")
    ap.add_argument("--stamps", action="store_true",
                    help="LNB fused, GRR_FUSED_STAMP build: print the per-phase s_memtime sums of each wave role")
    ap.add_argument("--mode", type=int, default=0, help="term: 0 GLR, 1 pair Laplacian, 2 prox")
    ap.add_argument("--width", type=int, default=0, help="image width (default: --size)")
    ap.add_argument("--acc", type=int, default=0, choices=[0, 1, 2],
                    help="term: 0 the term pass, 1 with the x-gradient pass inside (grr_bwd_term_fused_acc), "
                         "2 the term pass + the stencil x-gradient pass")
    ap.add_argument("--term-rows", type=int, default=2, choices=[0, 1, 2],
                    help="term: 0 per-pixel, 1 register-prefetch row kernel, 2 LDS-ring row kernel (default)")
    ap.add_argument("--c8", type=int, default=0, choices=[0, 1, 2, 3],
                    help="LNB fused: channel-blocked layout of x (1), out (2) or both (3)")
    args = ap.parse_args()
    K.set_kernel_variant(args.variant)
    K.set_term_rows(args.term_rows)
    from irdu_amd._native import call
    K.set_lnb_fused(bool(args.lnb_fused))
    dev = torch.device("cuda", 0)
    b, g, f, h, w = args.batch, args.graphs, args.fts, args.size, args.width or args.size
    c = g * f
    torch.manual_seed(0)
    mix = irdu_amd.MixtureGTVGLR(g, f, 0.5, 0.1, [[1e-3], [1e-4]], [[1e-4], [1e-4]], [[1e-4], [1e-4]],
                                 n_cgd_iters=10).to(dev)
    x = torch.rand(b, c, h, w, device=dev)
    rhs = torch.rand(b, c, h, w, device=dev)
    u = torch.rand(b, c, h, w, device=dev)
    th = torch.rand(b, c, h // 2, w // 2, device=dev)
    wl = torch.softmax(torch.rand(b, g, 4, h, w, device=dev), 2)
    cg = torch.rand(b, g, 2, h, w, device=dev)
    sl, sg = K.stencil(mix.GLRmodule00), K.stencil(mix.GTVmodule00)
    p = lambda t: t.data  # noqa: E731

    if args.kernel == "step":
        fn = lambda: K.system_step(x, rhs, u, th, wl, cg, sl, sg, p(mix.muys00), p(mix.ro00), p(mix.alphaCGD)[2],  # noqa: E731
                                   p(mix.betaCGD)[2], g, want_u=True, want_pool=True)
    elif args.kernel == "step2":
        wl1 = torch.softmax(torch.rand(b, g, 4, h // 2, w // 2, device=dev), 2)
        cg1 = torch.rand(b, g, 2, h // 2, w // 2, device=dev)
        sl1, sg1 = K.stencil(mix.GLRmodule01), K.stencil(mix.GTVmodule01)
        u_out = torch.empty_like(u)
        xd = torch.rand(b, c, h // 2, w // 2, device=dev)
        fn = lambda: K.system_step2(x, rhs, u, xd, wl, cg, sl, sg, p(mix.muys00), p(mix.ro00), wl1, cg1, sl1, sg1,  # noqa: E731
                                    p(mix.muys01), p(mix.ro01), p(mix.alphaCGD)[2], p(mix.betaCGD)[2],
                                    p(mix.alphaCGD)[3], p(mix.betaCGD)[3], g, want_u=True, want_pool=True,
                                    u_out=u_out)
    elif args.kernel == "half":
        xd = torch.rand(b, c, h // 2, w // 2, device=dev)
        wl1 = torch.softmax(torch.rand(b, g, 4, h // 2, w // 2, device=dev), 2)
        cg1 = torch.rand(b, g, 2, h // 2, w // 2, device=dev)
        fn = lambda: K.system_half(xd, wl1, cg1, sl, sg, p(mix.muys01), p(mix.ro01), g)  # noqa: E731
    elif args.kernel == "lnb":
        blk = irdu_amd.LocalNonLinearBlock(c, args.hid, 1).to(dev)
        if args.c8:   # the channel-blocked layout on the input (bit 0) / output (bit 1) side
            xin = K.to_c8(x) if args.c8 & 1 else x
            fn = lambda: blk._forward_c8(xin, bool(args.c8 & 1), bool(args.c8 & 2))  # noqa: E731
        else:
            fn = lambda: blk(x)  # noqa: E731
    elif args.kernel == "lnb_rep":   # first block of the image filter: RGB replicated over the graphs
        blk = irdu_amd.LocalNonLinearBlock(c, 256, 1).to(dev)
        src = torch.rand(b, 3, h, w, device=dev)
        ll, hid = blk.local_linear, 256
        wts = (p(blk.norm.weighted_transform.weight).view(c), p(ll.channels_linear_op.weight).view(2 * hid, c),
               p(ll.channels_local_linear_op.weight).view(2 * hid, 9), p(ll.project_out.weight).view(c, hid),
               p(blk.skip_weight))
        fn = lambda: K.lnb_forward_rep(src, None, *wts)  # noqa: E731
    elif args.kernel in ("feature_edges", "feature_edges_c8", "conv_edges"):   # a level's features -> edge weights
        wt = torch.rand(2 * c, c, 1, 1, device=dev) * 0.2
        mG, mL = torch.rand(g, f, device=dev) + 0.5, torch.rand(g, f, device=dev) + 0.5
        if args.kernel == "conv_edges":   # the two-pass path
            fn = lambda: K.edge_weights_block(K.conv1x1(x, wt), g, f, mG, mL)  # noqa: E731
        else:
            blocked = args.kernel.endswith("c8")
            xin = K.to_c8(x) if blocked else x
            fn = lambda: K.feature_edges(xin, blocked, wt, g, f, mG, mL)  # noqa: E731
    elif args.kernel == "conv1x1":
        wt = torch.rand(2 * c, c, 1, 1, device=dev)
        fn = lambda: K.conv1x1(x, wt)  # noqa: E731
    elif args.kernel == "conv_mk":     # conv1x1 at --cin -> --cout channels
        xk = torch.rand(b, args.cin, h, w, device=dev)
        wt = torch.rand(args.cout, args.cin, 1, 1, device=dev)
        fn = lambda: K.conv1x1(xk, wt)  # noqa: E731
    elif args.kernel == "conv_deep":   # the window FFBlock's W_in (K = 256 -> M = 1364), K-streaming x3 GEMM
        xd = torch.rand(b, 256, h, w, device=dev)
        wt = torch.rand(1364, 256, 1, 1, device=dev)
        fn = lambda: K.conv1x1(xd, wt)  # noqa: E731
    elif args.kernel == "term":   # the training reverse's operator-term pass (grr_bwd_term_fused)
        mode = args.mode
        gg = torch.randn(b, c, h, w, device=dev)
        taps = torch.randn(c, 5, device=dev) * 0.5
        wt = torch.rand(b, g, 2 if mode == 1 else 4, h, w, device=dev)
        lg = torch.log(torch.full((g,), 0.05, device=dev)) if mode == 2 else None
        sc = torch.rand(g, device=dev) + 0.5
        gw, gdot, gt = torch.zeros_like(wt), torch.zeros(g, device=dev), torch.zeros_like(taps)
        ggam = torch.zeros(g, device=dev) if mode == 2 else None
        gx = torch.zeros_like(x)
        if args.acc == 1:
            fn = lambda: K.bwd_term_fused_acc(mode, x, gg, taps, wt, lg, sc, 0.5, gx, gw, ggam, gdot, gt, g)  # noqa: E731
        elif args.acc == 2:
            fn = lambda: K.bwd_stencil(K.bwd_term_fused(mode, x, gg, taps, wt, lg, sc, 0.5, gw, ggam, gdot, gt, g),  # noqa: E731
                                       taps, K.ST_P_ADJ, g, sc, out=gx)
        else:
            fn = lambda: K.bwd_term_fused(mode, x, gg, taps, wt, lg, sc, 0.5, gw, ggam, gdot, gt, g)  # noqa: E731
    elif args.kernel == "gate_dw3_bwd":   # LNB training reverse: gate + depthwise adjoint, hid = --fts
        hid = args.fts
        hh = torch.randn(b, 2 * hid, h, w, device=dev)
        gq = torch.randn(b, hid, h, w, device=dev)
        wdw = torch.randn(2 * hid, 1, 3, 3, device=dev)
        sc = torch.tensor([0.7], device=dev)
        gwdw, gdot = torch.zeros_like(wdw), torch.zeros(1, device=dev)
        fn = lambda: K.lnb_gate_dw3_bwd(None, gq, sc, hh, wdw, gwdw, gdot)  # noqa: E731
    elif args.kernel == "edge":
        feat = torch.rand(b, 2 * c, h, w, device=dev)
        fn = lambda: K.edge_weights(feat, 0, g, f, p(mix.GTVmodule00.multiM))  # noqa: E731
    else:
        raise SystemExit(f"unknown kernel {args.kernel}")
    with torch.no_grad():
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        timer = K.LaunchTimer()
        timer.split_lnb = args.split
        K.set_timer(timer)
        for _ in range(args.iters):
            fn()
        K.set_timer(None)
        for kind, v in timer.summary().items():
            print(f"{args.kernel}: {kind:16s} launches={v['launches']} mean={v['mean_ms']:.4f} ms "
                  f"algo={v['gbps']:.1f} GB/s bytes/launch={v['bytes_per_launch']:.4e}")
    if args.stamps:
        import ctypes
        import numpy as np
        lib = irdu_amd.load_native()
        buf = (ctypes.c_ulonglong * (1024 * 64))()
        assert lib.grr_lnb_fused_stamps(buf, 1024 * 64) == 0
        a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 8, 8).astype(np.float64)
        nwg = int((a.sum(axis=(1, 2)) > 0).sum())
        a = a[:nwg]
        prod = ["dma", "prologue", "gemm1", "h_store", "wait", "barrier"]
        cons = ["dma", "gate", "gemm2", "epilogue", "wait", "barrier"]
        for name, waves, labels in (("producer", slice(0, 4), prod), ("consumer", slice(4, 8), cons)):
            m = a[:, waves, :6].mean(axis=(0, 1))
            tot = m.sum()
            print(f"stamps {name} ({nwg} workgroups, cycles per wave per launch): total {tot:.0f} " +
                  " ".join(f"{l}={v:.0f} ({v / tot:.0%})" for l, v in zip(labels, m)))


if __name__ == "__main__":
    main()
