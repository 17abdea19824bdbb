"""Time grr_wgrad against the library GEMM (torch.matmul(...).sum(0)) at the training step's shapes,
and grr_conv1x1 at its reverse shapes (HIP events on the current stream, median of 20)."""
import sys
import torch

sys.path.insert(0, ".")
import irdu_amd  # noqa: E402
from irdu_amd import kernels as K  # noqa: E402


def t(fn, n=20):
    for _ in range(3):
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
B = 16
for (m, k, hw) in [(512, 96, 256), (96, 256, 256), (192, 96, 256), (512, 96, 128), (96, 256, 128), (96, 384, 128),
                   (24, 96, 128)]:
    a = torch.randn(B, m, hw, hw, device=dev)
    x = torch.randn(B, k, hw, hw, device=dev)
    tw = t(lambda: K.wgrad(a, x))
    tl = t(lambda: torch.matmul(a.reshape(B, m, -1), x.reshape(B, k, -1).transpose(1, 2)).sum(0))
    gb = 4 * B * hw * hw * (m + k) / 1e9
    tf = 2 * B * hw * hw * m * k / 1e12
    print(f"wgrad {m}x{k} {B}x{hw}^2: grr {tw:.3f} ms ({gb / tw:.2f} TB/s, {tf / tw * 1e3:.0f} TF/s)  lib {tl:.3f} ms", flush=True)
for (k, m, hw) in [(96, 512, 256), (96, 256, 256), (512, 96, 256), (256, 96, 256), (192, 96, 256), (96, 192, 256),
                   (256, 1364, 256), (682, 256, 256)]:
    x = torch.randn(B, k, hw, hw, device=dev)
    w = torch.randn(m, k, 1, 1, device=dev)
    tc = t(lambda: K.conv1x1(x, w))
    gb = 4 * B * hw * hw * (m + k) / 1e9
    tf = 2 * B * hw * hw * m * k / 1e12
    print(f"conv1x1 {k}->{m} {B}x{hw}^2: {tc:.3f} ms ({gb / tc:.2f} TB/s, {tf / tc * 1e3:.0f} TF/s)", flush=True)
