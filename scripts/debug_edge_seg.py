"""Edge-weight row kernel: full batch vs one patch alone (bit-exact expected); prints the
first differing (output, graph, plane, row) per output when they differ."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import irdu_amd  # noqa: E402
from irdu_amd import kernels as K  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
for (b, h) in ((64, 256), (64, 128)):
    g, f = 32, 3
    feat = torch.randn(b, 2 * g * f, h, h, device=dev)
    mg = torch.rand(g, f, device=dev) + 0.5
    ml = torch.rand(g, f, device=dev) + 0.5
    full = K.edge_weights_block(feat, g, f, mg, ml)
    one = K.edge_weights_block(feat[1:2].contiguous(), g, f, mg, ml)
    for name, a, o in zip(("wG", "cG", "wL"), full, one):
        d = (a[1] - o[0]).abs()
        if d.max() == 0:
            print(h, name, "equal")
            continue
        idx = torch.nonzero(d)
        rows = sorted(set(idx[:, 2].tolist()))
        print(h, name, "max", float(d.max()), "n", idx.shape[0], "planes", sorted(set(idx[:, 1].tolist()))[:8],
              "rows", rows[:20])
