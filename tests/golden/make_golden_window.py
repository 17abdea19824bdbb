"""Golden vectors for the window-graph MixtureGTV by running the REFERENCE (build container only).

Usage:  python tests/golden/make_golden_window.py [--ref /root/reference]

Imports REF7 = exploration/model_multiscale_mixture_GLR/lib/model_GLR_GTV_deep_v7.py
read-only (no bytecode), builds its modules with seeded weights, moves the solver
scalars away from their near-zero inits so every term is exercised, and stores inputs,
``state_dict`` tensors and outputs as ``.npz`` data (no reference source):

  window_ops_v7.npz   GLRFast / GTVFast.extract_edge_weights + forward (REF7:274-782) on the
                      3x3 ring (K=8), the 5x5 diamond (K=12) and the full 5x5 window (K=24)
  window_v7.npz       MixtureGTV forward (REF7:802-1016; small CNN width) + its solver input
                      (features, y~) and the solver's graph-mixed output
  window_v1.npz       REF1 = lib/model_GLR_GTV_deep_v1.py MixtureGTV blocks (:472-676: 3x3 ring and full
                      5x5 window, no stats stencils, 6 CG stages) + SharpeningBlock (:768-787) forwards
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))

WINDOWS = {
    "ring3": np.array([1, 1, 1, 1, 0, 1, 1, 1, 1]).reshape(3, 3),
    "diamond5": np.array([0, 0, 1, 0, 0, 0, 1, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 1, 0, 0, 0, 1, 0, 0]).reshape(5, 5),
    "full5": np.array([1] * 12 + [0] + [1] * 12).reshape(5, 5),
}


def _import_v7(ref_root: str):
    sys.dont_write_bytecode = True
    sys.path.insert(0, os.path.join(ref_root, "exploration", "model_multiscale_mixture_GLR", "lib"))
    import model_GLR_GTV_deep_v7 as v7  # noqa: E402
    return v7


def _np(t):
    return t.detach().cpu().numpy().astype(np.float32)


def _perturb(mod, gen):
    with torch.no_grad():
        mod.stats_kernel_p01.copy_(0.8 + 0.4 * torch.rand(1, generator=gen))
        mod.stats_kernel_p02a.copy_(0.2 + 0.6 * torch.rand(1, generator=gen))
        mod.stats_kernel_p02b.copy_(0.2 + 0.6 * torch.rand(1, generator=gen))
        mod.stats_kernel_p03.copy_(0.1 + 0.5 * torch.rand(1, generator=gen))
        mod.multiM.copy_(0.5 + torch.rand(mod.multiM.shape, generator=gen))


def make_ops(v7, gen):
    out = {}
    b, g, f, fs, h, w = 2, 2, 3, 3, 12, 20
    for name, cw in WINDOWS.items():
        glr = v7.GLRFast(fs, f, g, cw, "cpu", M_diag_init=1.0)
        gtv = v7.GTVFast(fs, f, g, cw, "cpu", M_diag_init=1.0)
        _perturb(glr, gen)
        _perturb(gtv, gen)
        feat = torch.randn((b, g, f, h, w), generator=gen)
        x = torch.randn((b, g, fs, h, w), generator=gen)
        with torch.no_grad():
            wl, dl = glr.extract_edge_weights(feat)
            wg, dg = gtv.extract_edge_weights(feat)
            out[f"{name}/feat"] = _np(feat)
            out[f"{name}/x"] = _np(x)
            out[f"{name}/wL"] = _np(wl)
            out[f"{name}/wG"] = _np(wg)
            out[f"{name}/degL"] = _np(dl)
            out[f"{name}/glr"] = _np(glr(x, wl, dl))
            out[f"{name}/gtv"] = _np(gtv(x, wg, dg))
            out[f"{name}/gtv_C"] = _np(gtv.op_C(x, wg, dg))
        out[f"{name}/delta"] = np.asarray(glr.edge_delta, dtype=np.int32)
        for pre, mod in (("glr.", glr), ("gtv.", gtv)):
            for k, v in mod.state_dict().items():
                out[f"{name}/p/{pre}{k}"] = _np(v)
    np.savez_compressed(os.path.join(HERE, "window_ops_v7.npz"), **out)


def make_mixture(v7, gen):
    torch.manual_seed(2207)
    g, f = 4, 3
    cw = WINDOWS["diamond5"]
    mix = v7.MixtureGTV(nchannels_in=3, n_graphs=g, n_node_fts=f, n_cnn_fts=8, connection_window=cw, n_cgd_iters=4,
                        alpha_init=0.5, beta_init=0.1, muy_init=torch.tensor([[0.1], [0.0], [0.0], [0.0]]),
                        ro_init=torch.tensor([[0.1], [0.0], [0.0], [0.0]]),
                        gamma_init=torch.tensor([[0.001], [0.0], [0.0], [0.0]]), device="cpu")
    with torch.no_grad():
        mix.alphaCGD.copy_(0.2 + 0.6 * torch.rand(mix.alphaCGD.shape, generator=gen))
        mix.betaCGD.copy_(0.05 + 0.35 * torch.rand(mix.betaCGD.shape, generator=gen))
        mix.muys00.copy_(0.1 + 0.5 * torch.rand(mix.muys00.shape, generator=gen))
        mix.ro00.copy_(0.1 + 0.5 * torch.rand(mix.ro00.shape, generator=gen))
        mix.gamma00.copy_(torch.log(0.002 + 0.01 * torch.rand(mix.gamma00.shape, generator=gen)))
    _perturb(mix.GLRmodule00, gen)
    _perturb(mix.GTVmodule00, gen)
    clean = torch.rand((2, 3, 24, 40), generator=gen)
    noisy = clean + torch.randn(clean.shape, generator=gen) * (25.0 / 255.0)
    out = {"in/noisy": _np(noisy)}
    with torch.no_grad():
        feats = mix.patchs_features_extraction(noisy)[0]
        out["out/feats"] = _np(feats)
        out["out/dc"] = _np(mix.dc_estimator(feats[:, -12:]))
        out["out/y"] = _np(mix(noisy))
    for k, v in mix.state_dict().items():
        out["p/" + k] = _np(v)
    out["meta/n_state_keys"] = np.array(len(mix.state_dict()))
    np.savez_compressed(os.path.join(HERE, "window_v7.npz"), **out)


def _import_v1(ref_root: str):
    sys.dont_write_bytecode = True
    sys.path.insert(0, os.path.join(ref_root, "exploration", "model_multiscale_mixture_GLR", "lib"))
    import model_GLR_GTV_deep_v1 as v1  # noqa: E402
    return v1


def make_blocks_v1(v1, gen):
    """Two REF1 MixtureGTV blocks (3x3 ring K=8, full 5x5 K=24; 6 CG stages) + a SharpeningBlock at small
    widths (the full MultiScaleSequenceDenoiser's state_dict is 30 MB; its composition is checked
    against the oracle, which these blocks pin)."""
    torch.manual_seed(2201)
    out = {}
    for name, g, f, cw in (("ring3", 2, 3, WINDOWS["ring3"]), ("full5", 2, 2, WINDOWS["full5"])):
        mix = v1.MixtureGTV(nchannels_in=3, n_graphs=g, n_node_fts=f, connection_window=cw, n_cgd_iters=6,
                            alpha_init=0.5, beta_init=0.1, muy_init=torch.tensor([[0.1], [0.0], [0.0], [0.0]]),
                            ro_init=torch.tensor([[0.1], [0.0], [0.0], [0.0]]),
                            gamma_init=torch.tensor([[0.001], [0.0], [0.0], [0.0]]), device="cpu")
        with torch.no_grad():
            mix.alphaCGD.copy_(0.2 + 0.6 * torch.rand(mix.alphaCGD.shape, generator=gen))
            mix.betaCGD.copy_(0.05 + 0.35 * torch.rand(mix.betaCGD.shape, generator=gen))
            mix.muys00.copy_(0.1 + 0.5 * torch.rand(mix.muys00.shape, generator=gen))
            mix.ro00.copy_(0.1 + 0.5 * torch.rand(mix.ro00.shape, generator=gen))
            mix.gamma00.copy_(torch.log(0.002 + 0.01 * torch.rand(mix.gamma00.shape, generator=gen)))
            for mod in (mix.GLRmodule00, mix.GTVmodule00):
                mod.multiM.copy_(0.5 + torch.rand(mod.multiM.shape, generator=gen))
        clean = torch.rand((2, 3, 24, 40), generator=gen)
        noisy = clean + torch.randn(clean.shape, generator=gen) * (25.0 / 255.0)
        with torch.no_grad():
            out[f"{name}/in"] = _np(noisy)
            out[f"{name}/out"] = _np(mix(noisy))
        for k, v in mix.state_dict().items():
            out[f"{name}/p/{k}"] = _np(v)
        out[f"{name}/meta/n_state_keys"] = np.array(len(mix.state_dict()))
    sharp = v1.SharpeningBlock(3, 3, 24)
    with torch.no_grad():
        sharp.skip_connect_weight.copy_(torch.tensor([0.3, 0.8]))
        x = torch.rand((1, 3, 16, 20), generator=gen)
        out["sharp/in"] = _np(x)
        out["sharp/out"] = _np(sharp(x))
    for k, v in sharp.state_dict().items():
        out["sharp/p/" + k] = _np(v)
    np.savez_compressed(os.path.join(HERE, "window_v1.npz"), **out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    v7 = _import_v7(args.ref)
    gen = torch.Generator().manual_seed(2207)
    make_ops(v7, gen)
    make_mixture(v7, gen)
    make_blocks_v1(_import_v1(args.ref), torch.Generator().manual_seed(2201))
    for fn in ("window_ops_v7.npz", "window_v7.npz", "window_v1.npz"):
        print(fn, os.path.getsize(os.path.join(HERE, fn)))


if __name__ == "__main__":
    main()
