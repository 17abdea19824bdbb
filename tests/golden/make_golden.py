"""Generate golden vectors by running the REFERENCE implementation (build container only).

Usage:  python tests/golden/make_golden.py [--ref /root/reference]

Imports the reference modules read-only (bytecode writing disabled), builds them
with seeded weights, perturbs the scalar/solver parameters away from their
near-zero inits (so every term of the solver is exercised), runs them on seeded
synthetic inputs, and stores inputs, ``state_dict`` tensors and outputs as small
``.npz`` fixtures next to this script.  Only data is stored — no reference source.

Fixtures:
  ops_small.npz       GLRFast / GTVFast / soft-threshold / neighbour table (REF:13-523, :684-704)
  mixture_v1.npz      MixtureGTVGLR v1.0 forward + A(x) + L1-loss gradients (REF:526-811)
  mixture_v1_rect.npz same on a non-square, non-multiple-of-32 image
  msgf_v13.npz        v13_no_latent MultiScaleGraphFilter forward (lib/..._v13_no_latent.py:887-926)
  abstract_v1.npz     AbtractMultiScaleGraphFilter (small dims) forward + filtering (REF:1028-1174)
  mixture_glr_v10.npz / mixture_glr_v10_f1.npz
                      GLR-only MixtureGLR (lib/model_GLR_GTV_deep_v10.py:241-335) forward + L1 gradients
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def _import_ref(ref_root: str):
    sys.dont_write_bytecode = True
    v1_dir = os.path.join(ref_root, "exploration", "GGTV_GGLR_v1.0")
    lib_dir = os.path.join(ref_root, "exploration", "model_multiscale_mixture_GLR", "lib")
    sys.path.insert(0, v1_dir)
    sys.path.insert(0, lib_dir)
    import deep_multiscale_GGLR_GGTV_v1x0 as v1  # noqa: E402
    import model_GLR_GTV_deep_v13_no_latent as v13  # noqa: E402
    return v1, v13


def _import_v10(ref_root: str):
    sys.dont_write_bytecode = True
    sys.path.insert(0, os.path.join(ref_root, "exploration", "model_multiscale_mixture_GLR", "lib"))
    import model_GLR_GTV_deep_v10 as v10  # noqa: E402
    return v10


def make_mixture_glr(v10, gen, name, shape, g):
    b, c, h, w = shape
    mix = v10.MixtureGLR(n_graphs=g, n_node_fts=c // g, alpha_init=0.5, beta_init=0.1,
                         muy_init=torch.tensor([[0.001], [0.0], [0.0], [0.0]]))
    with torch.no_grad():
        mix.alphaCGD.copy_(0.2 + 0.6 * torch.rand(mix.alphaCGD.shape, generator=gen))
        mix.betaCGD.copy_(0.05 + 0.35 * torch.rand(mix.betaCGD.shape, generator=gen))
        mix.muys00.copy_(0.05 + 0.55 * torch.rand(mix.muys00.shape, generator=gen))
    _perturb_graph_module(mix.GLRmodule00, gen)
    x = torch.randn(shape, generator=gen) * 0.5 + 0.5
    target = torch.randn(shape, generator=gen) * 0.1
    out = {"in/x": _np(x), "in/target": _np(target), "meta/n_graphs": np.array(g)}
    _state(out, mix)
    with torch.no_grad():
        out["out/y"] = _np(mix(x))
    xg = x.clone().requires_grad_(True)
    loss = torch.nn.functional.l1_loss(mix(xg), target)
    loss.backward()
    out["grad/x"] = _np(xg.grad)
    for k, p in mix.named_parameters():
        out["grad/" + k] = _np(p.grad)
    np.savez_compressed(os.path.join(HERE, name), **out)


def _np(t: torch.Tensor) -> np.ndarray:
    return t.detach().cpu().numpy().copy()


def _perturb_graph_module(mod, gen: torch.Generator):
    with torch.no_grad():
        for nm in ("stats_kernel_p01", "stats_kernel_p02a", "stats_kernel_p02b", "stats_kernel_p03"):
            p = getattr(mod, nm)
            p.copy_(p * (1.0 + 0.25 * torch.randn(p.shape, generator=gen)))
        mod.multiM.copy_(1.0 + 0.3 * torch.randn(mod.multiM.shape, generator=gen))


def _perturb_mixture(mix, gen: torch.Generator):
    """Move solver scalars to values where every term matters."""
    def u(shape, lo, hi):
        return lo + (hi - lo) * torch.rand(shape, generator=gen)
    with torch.no_grad():
        mix.alphaCGD.copy_(u(mix.alphaCGD.shape, 0.2, 0.8))
        mix.betaCGD.copy_(u(mix.betaCGD.shape, 0.05, 0.4))
        for nm in ("muys00", "muys01", "ro00", "ro01"):
            p = getattr(mix, nm)
            p.copy_(torch.log(u(p.shape, 0.05, 0.6)))
        for nm in ("gamma00", "gamma01"):
            p = getattr(mix, nm)
            p.copy_(torch.log(u(p.shape, 0.002, 0.05)))
        for m in (mix.GLRmodule00, mix.GLRmodule01, mix.GTVmodule00, mix.GTVmodule01):
            _perturb_graph_module(m, gen)


def _smooth_image(gen: torch.Generator, shape, sigma=25.0):
    """Piecewise-smooth clean image in [0,1] + Gaussian noise (sigma/255)."""
    b, c, h, w = shape
    yy = torch.linspace(0, 1, h)[:, None]
    xx = torch.linspace(0, 1, w)[None, :]
    imgs = []
    for _ in range(b):
        chans = []
        for _ in range(c):
            fy, fx, ph = (torch.rand(3, generator=gen) * torch.tensor([4.0, 4.0, 6.28])).tolist()
            base = 0.5 + 0.3 * torch.sin(fy * 6.28 * yy + ph) * torch.cos(fx * 6.28 * xx)
            r0, c0 = int(torch.randint(0, h // 2, (1,), generator=gen)), int(torch.randint(0, w // 2, (1,), generator=gen))
            base[r0:r0 + h // 3, c0:c0 + w // 3] += 0.25
            chans.append(base)
        imgs.append(torch.stack(chans))
    clean = torch.stack(imgs).clamp(0, 1)
    clean = torch.round(clean * 255.0) / 255.0
    noisy = clean + torch.randn(clean.shape, generator=gen) * (sigma / 255.0)
    return clean.float(), noisy.float()


def _state(prefix_dict, module, prefix=""):
    for k, v in module.state_dict().items():
        prefix_dict["p/" + prefix + k] = _np(v)


def make_ops(v1, gen):
    out = {}
    b, g, f, h, w = 2, 2, 3, 16, 20
    glr = v1.GLRFast(n_node_fts=f, n_graphs=g, M_diag_init=1.0)
    gtv = v1.GTVFast(n_node_fts=f, n_graphs=g, M_diag_init=1.0)
    _perturb_graph_module(glr, gen)
    _perturb_graph_module(gtv, gen)
    feat = torch.randn(b, g, f, h, w, generator=gen)
    x = torch.randn(b, g, f, h, w, generator=gen)
    out["in/feat"] = _np(feat)
    out["in/x"] = _np(x)
    _state(out, glr, "glr.")
    _state(out, gtv, "gtv.")
    with torch.no_grad():
        wl, dl = glr.extract_edge_weights(feat)
        wg, dg = gtv.extract_edge_weights(feat)
        out["out/glr_w"], out["out/glr_deg"] = _np(wl), _np(dl)
        out["out/gtv_w"], out["out/gtv_deg"] = _np(wg), _np(dg)
        out["out/glr_stats_conv"] = _np(glr.stats_conv(x))
        out["out/glr_stats_conv_t"] = _np(glr.stats_conv_transpose(x))
        out["out/glr_op_L_norm"] = _np(glr.op_L_norm(x, wl, dl))
        out["out/glr_forward"] = _np(glr(x, wl, dl))
        e = gtv.op_C(x, wg, dg)
        out["out/gtv_op_C"] = _np(e)
        out["out/gtv_op_C_transpose"] = _np(gtv.op_C_transpose(e, wg, dg))
        out["out/gtv_forward"] = _np(gtv(x, wg, dg))
        # neighbour table: gather an index image through the reference's own gather
        idx = torch.arange(h * w, dtype=torch.float32).view(1, 1, h, w)
        nb = glr.get_neighbors_pixels(idx)  # [1,1,4,h,w]
        out["out/neighbor_table"] = nb[0, 0].to(torch.int32).numpy()
        out["out/edge_delta"] = glr.edge_delta.numpy()
    np.savez_compressed(os.path.join(HERE, "ops_small.npz"), **out)


def make_mixture(v1, gen, name, shape, g):
    b, c, h, w = shape
    mix = v1.MixtureGTVGLR(
        n_graphs=g, n_node_fts=c // g, alpha_init=0.5, beta_init=0.1,
        muy_init=torch.tensor([[0.001], [0.0001]]),
        ro_init=torch.tensor([[0.0001], [0.0001]]),
        gamma_init=torch.tensor([[0.0001], [0.0001]]))
    _perturb_mixture(mix, gen)
    x = torch.randn(shape, generator=gen) * 0.5 + 0.5
    target = torch.randn(shape, generator=gen) * 0.1
    out = {"in/x": _np(x), "in/target": _np(target), "meta/n_graphs": np.array(g)}
    _state(out, mix)
    with torch.no_grad():
        y = mix(x)
        # the system operator A applied to x, with this block's graphs (REF:642-682)
        f0 = mix.patchs_features_extraction00(x)
        f1 = mix.patchs_features_extraction01(x)
        a, bb = f0.chunk(2, dim=1)
        a1, b1 = f1.chunk(2, dim=1)
        gtv0 = mix.GTVmodule00.extract_edge_weights(a.reshape(b, g, c // g, h, w))
        glr0 = mix.GLRmodule00.extract_edge_weights(bb.reshape(b, g, c // g, h, w))
        gtv1 = mix.GTVmodule01.extract_edge_weights(a1.reshape(b, g, c // g, h // 2, w // 2))
        glr1 = mix.GLRmodule01.extract_edge_weights(b1.reshape(b, g, c // g, h // 2, w // 2))
        ax = mix.apply_lightweight_transformer(x.reshape(b, g, c // g, h, w), [gtv0, gtv1], [glr0, glr1])
    out["out/y"] = _np(y)
    out["out/Ax"] = _np(ax.reshape(shape))
    xg = x.clone().requires_grad_(True)
    loss = torch.nn.functional.l1_loss(mix(xg), target)
    loss.backward()
    out["out/loss"] = np.array(float(loss))
    out["grad/x"] = _np(xg.grad)
    for k, p in mix.named_parameters():
        out["grad/" + k] = _np(p.grad)
    np.savez_compressed(os.path.join(HERE, name), **out)


def make_msgf(v13, gen):
    g = 4
    model = v13.MultiScaleGraphFilter(n_channels_in=3, n_channels_out=3, ngraphs=g)
    _perturb_mixture(model.localfilter, gen)
    clean, noisy = _smooth_image(gen, (2, 3, 32, 32))
    out = {"in/noisy": _np(noisy), "in/clean": _np(clean), "meta/n_graphs": np.array(g)}
    _state(out, model)
    with torch.no_grad():
        out["out/y"] = _np(model(noisy))
    np.savez_compressed(os.path.join(HERE, "msgf_v13.npz"), **out)


def make_abstract(v1, gen):
    cfg = dict(n_channels_in=3, n_channels_out=3, dims=[8, 16, 32, 64], hidden_dims=[16, 24, 32, 48],
               nsubnets=[1, 1, 1, 1], ngraphs=[2, 4, 4, 8], num_blocks=[1, 1, 1, 1], num_blocks_out=1)
    model = v1.AbtractMultiScaleGraphFilter(**cfg)
    for blk in (model.localfilter_scale_00, model.localfilter_scale_01,
                model.localfilter_scale_02, model.localfilter_scale_03):
        _perturb_mixture(blk.local_filter, gen)
    clean, noisy = _smooth_image(gen, (1, 3, 32, 32))
    out = {"in/noisy": _np(noisy), "in/clean": _np(clean)}
    for k, v in cfg.items():
        out["meta/" + k] = np.array(v)
    _state(out, model)
    with torch.no_grad():
        coefs = model.encode(noisy)
        filt = model.filtering(coefs)
        out["out/y"] = _np(model(noisy))
        for i in range(4):
            out[f"out/coef{i}"] = _np(coefs[i])
            out[f"out/filtered{i}"] = _np(filt[i])
    out["meta/n_state_keys"] = np.array(len(model.state_dict()))
    np.savez_compressed(os.path.join(HERE, "abstract_v1.npz"), **out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", choices=["all", "v10"], default="all")
    args = ap.parse_args()
    if args.only in ("all", "v10"):   # own generator: (re)making these leaves the others untouched
        v10 = _import_v10(args.ref)
        gen10 = torch.Generator().manual_seed(2210)
        make_mixture_glr(v10, gen10, "mixture_glr_v10.npz", (2, 12, 24, 32), 4)
        make_mixture_glr(v10, gen10, "mixture_glr_v10_f1.npz", (1, 8, 20, 28), 8)
        if args.only == "v10":
            return
    v1, v13 = _import_ref(args.ref)
    torch.manual_seed(2204)
    gen = torch.Generator().manual_seed(2204)
    make_ops(v1, gen)
    make_mixture(v1, gen, "mixture_v1.npz", (2, 12, 32, 32), 4)
    make_mixture(v1, gen, "mixture_v1_rect.npz", (1, 12, 24, 40), 2)
    make_msgf(v13, gen)
    make_abstract(v1, gen)
    for fn in sorted(os.listdir(HERE)):
        if fn.endswith(".npz"):
            print(fn, os.path.getsize(os.path.join(HERE, fn)))


if __name__ == "__main__":
    main()
