"""Window term reverses with the E / PW planes (pass 1 writes, pass 2 gathers) against the fused gather
(kernels.WIN_FUSED_GATHER): ms per call at B x G x Fs x H x W with K-edge windows (HIP events)."""
import sys

import torch

sys.path.insert(0, ".")
import irdu_amd  # noqa: E402
from irdu_amd import kernels as K  # noqa: E402
import numpy as np  # noqa: E402

irdu_amd.load_native()
dev = "cuda:0"
B, G, Fs, H, W = 4, 8, 3, 256, 256
for name, cw in (("ring5", np.ones((5, 5))), ("ring3", np.ones((3, 3)))):
    cw = cw.copy()
    cw[cw.shape[0] // 2, cw.shape[1] // 2] = 0
    m = np.arange(cw.shape[0]) - cw.shape[0] // 2
    dl = tuple((int(dy), int(dx)) for i, dy in enumerate(m) for j, dx in enumerate(m) if cw[i, j])
    k = len(dl)
    s = torch.randn(B, G, Fs, H, W, device=dev)
    bt = torch.randn_like(s)
    wt = torch.softmax(torch.randn(B, G, k, H, W, device=dev), 2)
    sc = torch.rand(G, device=dev) + 0.2
    lg = torch.log(torch.full((G,), 0.1, device=dev))
    gw = torch.zeros_like(wt)
    gdot, ggam = torch.zeros(G, device=dev), torch.zeros(G, device=dev)
    for term in ("glr", "prox"):
        res = {}
        for fused in (False, True):
            K.WIN_FUSED_GATHER = fused
            fn = (lambda: K.win_bwd_glr(s, bt, wt, dl, sc, -1.0, gw, gdot, G)) if term == "glr" else \
                (lambda: K.win_bwd_gtv(s, bt, wt, dl, True, lg, sc, 1.0, gw, gdot, ggam, G))
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[fused] = e0.elapsed_time(e1) / 10
        print(f"{name} K={k} {term}: planes {res[False]:.3f} ms  fused {res[True]:.3f} ms  x{res[False] / res[True]:.2f}",
              flush=True)
