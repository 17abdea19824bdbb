import sys, os, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import irdu_amd
from oracle import graph_oracle as O
def run(shape, which):
    torch.manual_seed(0)
    b, g, f, h, w = shape
    x = torch.randn(b, g, f, h, w)
    wt = torch.softmax(torch.randn(b, g, 4, h, w), 2)
    m = (irdu_amd.GLRFast if which == "glr" else irdu_amd.GTVFast)(f, g, 1.0)
    k = O.stats_kernel({kk: v.detach() for kk, v in m.state_dict().items()}, "")
    ref = (O.glr_apply if which == "glr" else O.gtv_apply)(x, wt, k)
    m = m.cuda()
    with torch.no_grad():
        out = m(x.cuda(), wt.cuda()).cpu()
    err = (out - ref).abs()
    scale = ref.abs().max()
    print(which, shape, "rel", float(err.max() / scale))
    e = err.reshape(b * g * f, h, w)
    print("  per-plane", [round(float(v / scale), 4) for v in e.flatten(1).max(1).values])
    print("  per-row", [round(float(v / scale), 3) for v in e.max(0).values.max(1).values])
    print("  per-col", [round(float(v / scale), 3) for v in e.max(0).values.max(0).values])
for which in ("glr", "gtv"):
    for shape in [(1, 1, 1, 8, 70), (1, 1, 2, 8, 20), (1, 2, 1, 8, 20), (2, 1, 1, 8, 20), (1, 1, 1, 70, 20)]:
        run(shape, which)
