"""Which kernel breaks bitwise batch independence: the fused LNB (C8 in) and feature_edges, batch 64 vs slices."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
import irdu_amd
from irdu_amd import kernels as K

irdu_amd.load_native()
dev = torch.device("cuda", 0)
torch.manual_seed(3)
B, G, H, W = 64, 32, 256, 256
c = 3 * G
x = (torch.randn(B, c, H, W) * torch.rand(B, 1, H, W) * 3).to(dev)
wt = (torch.randn(2 * c, c, 1, 1) * 0.2).to(dev)
mG = (0.5 + torch.rand(G, 3)).to(dev)
mL = (0.5 + torch.rand(G, 3)).to(dev)
for blocked in (False, True):
    xin = K.to_c8(x) if blocked else x
    full = K.feature_edges(xin, blocked, wt, G, 3, mG, mL)
    for i in (0, 17, 63):
        xi = K.to_c8(x[i:i + 1].contiguous()) if blocked else x[i:i + 1].contiguous()
        one = K.feature_edges(xi, blocked, wt, G, 3, mG, mL)
        for name, f, o in zip(("wG", "cG", "wL"), full, one):
            d = (f[i] - o[0]).abs()
            if d.max().item() != 0:
                idx = (d == d.max()).nonzero()[0].tolist()
                print("feature_edges blocked", blocked, "item", i, name, "maxdiff", d.max().item(), "at", idx,
                      "n diff", int((d != 0).sum()))
print("feature_edges done")
blk = irdu_amd.LocalNonLinearBlock(c, 256, 1).to(dev)
with torch.no_grad():
    for p in blk.parameters():
        p.add_(torch.randn_like(p) * 0.05)
    full = blk(x)
    for i in (0, 17, 63):
        one = blk(x[i:i + 1].contiguous())
        d = (full[i] - one[0]).abs()
        if d.max().item() != 0:
            print("lnb item", i, "maxdiff", d.max().item(), "n diff", int((d != 0).sum()))
print("lnb done")
