"""grr_wgrad per-shape tile plan (grr_wgrad_set_tiles 1) against the 128 x 96 tile alone (0) at the v1.0
model's C4 shapes (512^2 x 32 and its levels): median of HIP-event times, TF/s on the algorithmic flops."""
import sys

import torch

sys.path.insert(0, ".")
import irdu_amd  # noqa: E402
from irdu_amd import kernels as K  # noqa: E402


def t(fn, n=10):
    for _ in range(2):
        fn()
    ts = []
    for _ in range(n):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(); fn(); e.record(); e.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]


irdu_amd.load_native()
dev = "cuda:0"
B = 32
for (m, k, hw) in [(192, 48, 512), (48, 96, 512), (96, 48, 512), (48, 192, 512), (384, 96, 256), (96, 192, 256),
                   (768, 192, 128), (192, 384, 128), (1536, 384, 64), (384, 768, 64)]:
    a = torch.randn(B, m, hw, hw, device=dev)
    x = torch.randn(B, k, hw, hw, device=dev)
    fl = 2.0 * B * m * k * hw * hw
    res = {}
    for tiles in (False, True):
        K.set_wgrad_tiles(tiles)
        res[tiles] = t(lambda: K.wgrad(a, x))
    K.set_wgrad_tiles(True)
    print(f"M={m:5d} K={k:4d} {hw}^2: 128x96 {res[False]:7.3f} ms ({fl / res[False] / 1e9:6.1f} TF/s)  "
          f"plan {res[True]:7.3f} ms ({fl / res[True] / 1e9:6.1f} TF/s)  x{res[False] / res[True]:.2f}", flush=True)
    del a, x
