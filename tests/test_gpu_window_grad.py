"""GPU parity of the window-graph training reverse (window_bwd.hip via irdu_amd.window_grad).

Every gradient is checked against PyTorch autograd through the CPU oracle
(oracle/window_oracle.py, float64; the oracle's forward is pinned to the reference's own
outputs by tests/test_oracle_golden.py): per operator term (GLR, linear GTV, prox GTV) on the
three windows the reference uses (3x3 ring K=8, 5x5 diamond K=12, full 5x5 K=24), the whole
unrolled solver, the mixture, a training step of the REF7 / REF1 MixtureGTV blocks, and the bare
GLRFast / GTVFast module calls (extract_edge_weights + forward) under autograd.
Tolerances: max-abs error / max-abs reference <= 2e-4 where every soft-threshold branch is
stable (gamma far from |C x| or tiny); relative L2 <= 2e-3 where a few of the millions of
|C x| ~ gamma comparisons may legitimately flip between fp32 and fp64.
"""
import math

import numpy as np
import pytest
import torch

from oracle import window_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
WINDOWS = {"ring3": np.array([1, 1, 1, 1, 0, 1, 1, 1, 1]).reshape(3, 3),
           "diamond5": np.array([0, 0, 1, 0, 0, 0, 1, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 1, 0, 0, 0, 1, 0, 0])
           .reshape(5, 5),
           "full5": np.array([1] * 12 + [0] + [1] * 12).reshape(5, 5)}


@pytest.fixture(scope="module")
def wg():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import irdu_amd
    irdu_amd.load_native()
    from irdu_amd import window_grad, window_graph, window_graph_v1
    return window_grad, window_graph, window_graph_v1


def rel_inf(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    assert a.shape == b.shape, (a.shape, b.shape)
    return float((a - b).abs().max()) / max(float(b.abs().max()), 1e-30)


def rel_l2(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    assert a.shape == b.shape, (a.shape, b.shape)
    return float((a - b).norm()) / max(float(b.norm()), 1e-30)


def _taps_params(gen):
    return {k: (lo + span * torch.rand(1, generator=gen, dtype=torch.float64))
            for k, lo, span in (("stats_kernel_p01", 0.8, 0.4), ("stats_kernel_p02a", 0.2, 0.6),
                                ("stats_kernel_p02b", 0.2, 0.6), ("stats_kernel_p03", 0.1, 0.5))}


def _weights(b, g, k, h, w, gen):
    return torch.softmax(2.0 * torch.randn((b, g, k, h, w), generator=gen, dtype=torch.float64), dim=2)


def _dev(t):
    return t.float().to(DEV).contiguous()


@pytest.mark.parametrize("hw", [(21, 37), (2, 3), (3, 2)])    # tiny frames: the clamp folds several pixels
@pytest.mark.parametrize("name", sorted(WINDOWS))
@pytest.mark.parametrize("term", ["glr", "gtv", "prox"])
def test_window_term_reverse_vs_oracle(wg, name, term, hw):
    """One operator term  coef * scale[g] * T(Z(P x)): x-gradient, weight, tap and scalar gradients."""
    WG = wg[0]
    cw = WINDOWS[name]
    delta = O.window_edges(cw)
    dl = tuple((int(a), int(c)) for a, c in delta)
    b, g, fs = 2, 3, 3
    h, w = hw
    gen = torch.Generator().manual_seed(77 + len(delta) + len(term))
    k = len(delta)
    x = torch.randn((b, g, fs, h, w), generator=gen, dtype=torch.float64)
    gg = torch.randn_like(x)
    wt = _weights(b, g, k, h, w, gen)
    tp = _taps_params(gen)
    scale = 0.2 + torch.rand(g, generator=gen, dtype=torch.float64)
    log_gamma = torch.log(0.05 + 0.1 * torch.rand(g, generator=gen, dtype=torch.float64))
    coef = -1.0 if term != "prox" else 1.0
    # oracle (autograd, float64)
    xr, wr, sr, lr = (t.clone().requires_grad_(True) for t in (x, wt, scale, log_gamma))
    tpr = {q: v.clone().requires_grad_(True) for q, v in tp.items()}
    kern = O.stats_kernel({"m." + q: v for q, v in tpr.items()}, "m.", fs)
    if term == "glr":
        y = O.glr_apply(xr, wr, kern, delta)
    else:
        e = O.gtv_C(xr, wr, kern, delta)
        if term == "prox":
            eps = O.soft_threshold(e, torch.exp(lr))
            e = eps - (e - eps)
        y = O.gtv_Ct(e, wr, kern, delta)
    (coef * (gg * y * sr[None, :, None, None, None]).sum()).backward()
    # HIP
    taps = WG.K.win_taps(*[_dev(tp[q]) for q in WG.STENCIL_PARAMS])
    T = WG._Terms(_dev(wt), _dev(wt), taps, taps, _dev(scale), _dev(scale), _dev(log_gamma), dl, g)
    out = torch.zeros((b, g, fs, h, w), device=DEV)
    if term == "glr":
        T.glr_bwd(_dev(x), _dev(gg), coef, out)
        gw, gsc, gt = T.gwL, T.gmu, T.gtL
    else:
        T.gtv_bwd(_dev(x), _dev(gg), coef, out, prox=term == "prox")
        gw, gsc, gt = T.gwG, T.gro, T.gtG
    torch.cuda.synchronize()
    assert rel_inf(out, xr.grad) <= 2e-4
    assert rel_inf(gw, wr.grad) <= 2e-4
    assert rel_inf(gsc, sr.grad) <= 2e-4
    gp = WG.taps_backward(gt)
    for q, v in zip(WG.STENCIL_PARAMS, gp):
        assert rel_inf(v, tpr[q].grad) <= 2e-4, q
    if term == "prox":
        assert rel_inf(T.ggam * torch.exp(_dev(log_gamma)), lr.grad) <= 2e-4


@pytest.mark.parametrize("hw", [(19, 33), (2, 5)])
@pytest.mark.parametrize("name", sorted(WINDOWS))
def test_window_edge_weight_reverse_vs_oracle(wg, name, hw):
    WG = wg[0]
    delta = O.window_edges(WINDOWS[name])
    dl = tuple((int(a), int(c)) for a, c in delta)
    b, g, f = 2, 3, 5
    h, w = hw
    gen = torch.Generator().manual_seed(91 + len(delta))
    feat = torch.randn((b, g * f + 4, h, w), generator=gen, dtype=torch.float64)
    feat[0, :f, min(3, h - 1), 4] = 0.0              # a zero-norm pixel (normalize's eps branch)
    M = 0.5 + torch.rand((g, f), generator=gen, dtype=torch.float64)
    gw_up = torch.randn((b, g, len(delta), h, w), generator=gen, dtype=torch.float64)
    fr, Mr = feat.clone().requires_grad_(True), M.clone().requires_grad_(True)
    wt, _ = O.edge_weights(fr[:, :g * f].reshape(b, g, f, h, w), Mr, delta)
    (wt * gw_up).sum().backward()
    fd = _dev(feat)
    wd, _ = WG.K.win_edge_weights(fd, 0, g, f, _dev(M), dl)
    assert rel_inf(wd, wt) <= 1e-5
    gfeat, gM = torch.zeros_like(fd), torch.zeros((g, f), device=DEV)
    WG.K.win_bwd_edge_weights(fd, 0, g, f, _dev(M), wd, _dev(gw_up), dl, gfeat, gM)
    torch.cuda.synchronize()
    mask = torch.ones_like(fr.grad, dtype=torch.bool)
    mask[0, :f, min(3, h - 1), 4] = False            # its gradient is scaled by 1 / eps: checked apart
    assert rel_inf(gfeat.cpu()[mask], fr.grad[mask]) <= 2e-4
    assert rel_inf(gfeat.cpu()[~mask], fr.grad[~mask]) <= 2e-4
    assert rel_inf(gM, Mr.grad) <= 2e-4


def _solver_params(g, f, iters, gen, gamma):
    d = torch.float64
    p = {"GTVmodule00.multiM": 0.5 + torch.rand((g, f), generator=gen, dtype=d),
         "GLRmodule00.multiM": 0.5 + torch.rand((g, f), generator=gen, dtype=d),
         "ro00": 0.1 + 0.5 * torch.rand(g, generator=gen, dtype=d),
         "muys00": 0.1 + 0.5 * torch.rand(g, generator=gen, dtype=d),
         "gamma00": torch.log(gamma * (1.0 + torch.rand(g, generator=gen, dtype=d))),
         "alphaCGD": 0.2 + 0.6 * torch.rand((iters, g), generator=gen, dtype=d),
         "betaCGD": 0.05 + 0.35 * torch.rand((iters, g), generator=gen, dtype=d)}
    for pre in ("GTVmodule00.", "GLRmodule00."):
        for q, v in _taps_params(gen).items():
            p[pre + q] = v
    return p


class _SolverHolder(torch.nn.Module):
    def __init__(self, wgm, p, g, f, iters, cw, taps):
        super().__init__()
        self.n_graphs, self.n_node_fts, self.n_cgd_iters = g, f, iters
        self.GTVmodule00 = wgm.GTVFast(3, f, g, cw)
        self.GLRmodule00 = wgm.GLRFast(3, f, g, cw)
        for k in ("ro00", "muys00", "gamma00", "alphaCGD", "betaCGD"):
            setattr(self, k, torch.nn.Parameter(p[k].float().clone()))
        for pre, mod in (("GTVmodule00.", self.GTVmodule00), ("GLRmodule00.", self.GLRmodule00)):
            mod.load_state_dict({k[len(pre):]: v.float() for k, v in p.items()
                                 if k.startswith(pre) and (taps or "stats" not in k)}, strict=taps)


@pytest.mark.parametrize("name,shape,iters,gamma,taps", [
    ("diamond5", (2, 4, 3, 24, 40), 4, 1e-9, True),
    ("ring3", (1, 3, 6, 30, 20), 6, 1e-9, True),
    ("full5", (1, 2, 4, 17, 29), 5, 1e-9, False),
    ("diamond5", (1, 2, 3, 16, 24), 4, 0.02, True),
])
def test_window_solver_reverse_vs_oracle(wg, name, shape, iters, gamma, taps):
    """The whole unrolled solver (rhs, 2 stages, prox rhs, stages 2..S-1): gradients of y, the
    features and every solver parameter vs oracle autograd."""
    WG, wgm, _ = wg
    b, g, f, h, w = shape
    cw = WINDOWS[name]
    delta = O.window_edges(cw)
    gen = torch.Generator().manual_seed(313 + h + iters)
    p = _solver_params(g, f, iters, gen, gamma)
    y = torch.rand((b, 3, h, w), generator=gen, dtype=torch.float64)
    feat = torch.randn((b, g * f + 2, h, w), generator=gen, dtype=torch.float64)
    gout = torch.randn((b, g, 3, h, w), generator=gen, dtype=torch.float64)
    names = WG.param_names(taps)
    pr = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    yr, fr = y.clone().requires_grad_(True), feat.clone().requires_grad_(True)
    ref = O.mixture_solve(yr, fr[:, :g * f], pr, g, f, delta, n_cgd_iters=iters, stats=taps)
    (ref * gout).sum().backward()

    mod = _SolverHolder(wgm, p, g, f, iters, cw, taps).to(DEV)
    yd, fd = _dev(y).requires_grad_(True), _dev(feat).requires_grad_(True)
    out = WG.window_solve(mod, yd, fd, with_taps=taps)
    assert rel_inf(out, ref) <= 1e-4
    (out * _dev(gout)).sum().backward()
    tol, metric = (2e-4, rel_inf) if gamma < 1e-6 else (2e-3, rel_l2)
    assert metric(yd.grad, yr.grad) <= tol
    assert metric(fd.grad, fr.grad) <= tol
    for n in names:
        got = WG._get(mod, n).grad
        assert got is not None, n
        if gamma < 1e-6 and n == "gamma00":
            continue                                   # ~0 when no edge reaches gamma
        assert metric(got, pr[n].grad) <= tol, n


def test_window_mix_reverse(wg):
    WG = wg[0]
    gen = torch.Generator().manual_seed(5)
    x = torch.randn((2, 5, 3, 9, 14), generator=gen)
    sc = torch.softmax(torch.randn((2, 5, 9, 14), generator=gen), dim=1)
    dc = torch.randn((2, 3, 9, 14), generator=gen)
    go = torch.randn((2, 3, 9, 14), generator=gen)
    xr, sr, dr = (t.clone().requires_grad_(True) for t in (x, sc, dc))
    (torch.einsum("bgchw, bghw -> bchw", xr, sr) + dr).mul(go).sum().backward()
    xd, sd, dd = (_dev(t).requires_grad_(True) for t in (x, sc, dc))
    WG.WinMixFn.apply(xd, sd, dd).mul(_dev(go)).sum().backward()
    assert rel_inf(xd.grad, xr.grad) <= 1e-6
    assert rel_inf(sd.grad, sr.grad) <= 1e-5
    assert rel_inf(dd.grad, dr.grad) == 0.0


def _model_grads_vs_oracle(model, oracle_fn, img, tol):
    p = {k: v.detach().clone().double().requires_grad_(True) for k, v in model.named_parameters()}
    gen = torch.Generator().manual_seed(9)
    go = torch.randn(img.shape, generator=gen, dtype=torch.float64)
    ref = oracle_fn(img.double(), p)
    (ref * go).sum().backward()
    model = model.to(DEV).train()
    out = model(img.to(DEV))
    assert rel_inf(out, ref) <= 1e-4
    (out * go.float().to(DEV)).sum().backward()
    for k, prm in model.named_parameters():
        assert prm.grad is not None, k
        if k.endswith("gamma00"):
            # gamma = 1e-9 keeps every soft-threshold branch stable; its own gradient is then ~0
            # on both sides (rounding noise) -- checked at gamma = 0.02 by the solver test
            assert float(prm.grad.abs().max()) <= 1e-6 * max(float(p[k.replace("gamma00", "ro00")].grad.abs().max()), 1)
            continue
        assert rel_l2(prm.grad, p[k].grad) <= tol, k


def test_window_v7_training_step_grads(wg):
    """MixtureGTV of REF7 (G=4, F=3, diamond K=12, 4 stages) trained end to end: every parameter's
    gradient (feature CNN, DC estimator, combination conv, solver) vs the oracle's autograd."""
    _, wgm, _ = wg
    torch.manual_seed(41)
    m = wgm.MixtureGTV(3, 4, 3, 8, wgm.CONNECTION_FLAGS_5x5_small, 4, 0.5, 0.1, torch.tensor([[0.3]]),
                       torch.tensor([[0.2]]), torch.tensor([[1e-9]]))
    img = torch.rand((2, 3, 24, 32))
    _model_grads_vs_oracle(m, lambda x, p: O.mixture_gtv_v7(x, p, 4, 3, wgm.CONNECTION_FLAGS_5x5_small), img, 2e-3)


def test_window_v1_training_step_grads(wg):
    """MixtureGTV of REF1 (identity stencil, K=8 ring, 6 stages) trained end to end."""
    _, wgm, W1 = wg
    torch.manual_seed(43)
    m = W1.MixtureGTV(3, 2, 3, wgm.CONNECTION_FLAGS_3x3, 6, 0.5, 0.1, torch.tensor([[0.3]]), torch.tensor([[0.2]]),
                      torch.tensor([[1e-9]]))
    img = torch.rand((1, 3, 16, 24))
    _model_grads_vs_oracle(m, lambda x, p: O.mixture_gtv_v1(x, p, 2, 3, wgm.CONNECTION_FLAGS_3x3), img, 2e-3)


@pytest.mark.parametrize("version", ["v7", "v1"])
@pytest.mark.parametrize("name", sorted(WINDOWS))
def test_window_module_calls_differentiable(wg, version, name):
    """The bare module calls of REF7 (:418-511, :776-782) / REF1 (:255-291, :421-470) under autograd:
    w = extract_edge_weights(features), then GLRFast.forward(x, w_L) and GTVFast.forward(x, w_G); the
    loss also reads the node degree.  Feature, signal, multiM and stats-stencil gradients vs the float64
    oracle's autograd (REF1: identity stencil, no stencil parameters)."""
    WG, W7, W1 = wg
    mod = W7 if version == "v7" else W1
    cw = WINDOWS[name]
    delta = O.window_edges(cw)
    b, g, f, fs, h, w = 2, 3, 4, 3, 17, 29
    gen = torch.Generator().manual_seed(301 + len(delta) + len(version))
    feat = torch.randn((b, g, f, h, w), generator=gen, dtype=torch.float64)
    x = torch.randn((b, g, fs, h, w), generator=gen, dtype=torch.float64)
    ggl, ggt = torch.randn_like(x), torch.randn_like(x)
    gd = torch.randn((b, g, h, w), generator=gen, dtype=torch.float64)
    ML = 0.5 + torch.rand((g, f), generator=gen, dtype=torch.float64)
    MG = 0.5 + torch.rand((g, f), generator=gen, dtype=torch.float64)
    tpl, tpg = _taps_params(gen), _taps_params(gen)
    glr = mod.GLRFast(fs, f, g, cw).to(DEV)
    gtv = mod.GTVFast(fs, f, g, cw).to(DEV)
    with torch.no_grad():
        glr.multiM.copy_(ML)
        gtv.multiM.copy_(MG)
        if version == "v7":
            for m_, tp in ((glr, tpl), (gtv, tpg)):
                for q, v in tp.items():
                    getattr(m_, q).copy_(v)
    # HIP
    fr, xr = _dev(feat).requires_grad_(True), _dev(x).requires_grad_(True)
    wl, degl = glr.extract_edge_weights(fr)
    wgt, _ = gtv.extract_edge_weights(fr)
    loss = (_dev(ggl) * glr(xr, wl, degl)).sum() + (_dev(ggt) * gtv(xr, wgt)).sum() + (_dev(gd) * degl).sum()
    loss.backward()
    torch.cuda.synchronize()
    # oracle (autograd, float64)
    fo, xo = feat.clone().requires_grad_(True), x.clone().requires_grad_(True)
    MLo, MGo = ML.clone().requires_grad_(True), MG.clone().requires_grad_(True)
    tlo = {q: v.clone().requires_grad_(True) for q, v in tpl.items()}
    tgo = {q: v.clone().requires_grad_(True) for q, v in tpg.items()}
    kl = O.stats_kernel({"m." + q: v for q, v in tlo.items()}, "m.", fs) if version == "v7" else None
    kg = O.stats_kernel({"m." + q: v for q, v in tgo.items()}, "m.", fs) if version == "v7" else None
    wlo, dlo = O.edge_weights(fo, MLo, delta)
    wgo, _ = O.edge_weights(fo, MGo, delta)
    ref = ((ggl * O.glr_apply(xo, wlo, kl, delta)).sum() + (ggt * O.gtv_Ct(O.gtv_C(xo, wgo, kg, delta), wgo, kg, delta)).sum()
           + (gd * dlo).sum())
    ref.backward()
    assert rel_inf(xr.grad, xo.grad) <= 2e-4
    assert rel_inf(fr.grad, fo.grad) <= 2e-4
    assert rel_inf(glr.multiM.grad, MLo.grad) <= 2e-4
    assert rel_inf(gtv.multiM.grad, MGo.grad) <= 2e-4
    if version == "v7":
        for m_, to in ((glr, tlo), (gtv, tgo)):
            for q, v in to.items():
                assert rel_inf(getattr(m_, q).grad, v.grad) <= 2e-4, q


@pytest.mark.parametrize("hw", [(21, 37), (2, 3), (3, 2), (64, 64)])
@pytest.mark.parametrize("name", sorted(WINDOWS))
@pytest.mark.parametrize("term", ["glr", "gtv", "prox", "prox_tiny"])
def test_window_fused_gather_equals_planes(wg, name, term, hw):
    """grr_win_bwd_gather_fused (the E / PW terms recomputed where they are gathered; pass 1 writes no
    planes) against pass 1 writing E / PW + grr_win_bwd_gather: l or o, gs, and the weight / scalar
    gradients pass 1 accumulates, to fp32 rounding (the same expressions in two kernels)."""
    K = wg[0].K
    delta = O.window_edges(WINDOWS[name])
    dl = tuple((int(a), int(c)) for a, c in delta)
    b, g, fs = 2, 3, 3
    h, w = hw
    k = len(delta)
    gen = torch.Generator().manual_seed(501 + k + len(term) + h)
    s = _dev(torch.randn((b, g, fs, h, w), generator=gen, dtype=torch.float64))
    bt = _dev(torch.randn((b, g, fs, h, w), generator=gen, dtype=torch.float64))
    wt = _dev(_weights(b, g, k, h, w, gen))
    sc = _dev(0.2 + torch.rand(g, generator=gen, dtype=torch.float64))
    lg = _dev(torch.log(0.05 + 0.5 * torch.rand(g, generator=gen, dtype=torch.float64)))
    if term == "prox_tiny":                     # gamma 1e-9: the soft threshold's branch at z = 0 matters
        lg = torch.full_like(lg, math.log(1e-9))
        term = "prox"
    res = {}
    saved = K.WIN_FUSED_GATHER
    try:
        for fused in (False, True):
            K.WIN_FUSED_GATHER = fused
            gw = torch.full_like(wt, 0.25)
            gdot = torch.zeros(g, device=DEV)
            ggam = torch.zeros(g, device=DEV)
            if term == "glr":
                out = K.win_bwd_glr(s, bt, wt, dl, sc, -1.0, gw, gdot, g)
            else:
                out = K.win_bwd_gtv(s, bt, wt, dl, term == "prox", lg if term == "prox" else None, sc, 1.0, gw, gdot,
                                    ggam if term == "prox" else None, g)
            torch.cuda.synchronize()
            res[fused] = [t.cpu() for t in (*out, gw, gdot, ggam)]
    finally:
        K.WIN_FUSED_GATHER = saved
    for nm, a, r in zip(("l/o", "gs", "gw", "gdot", "ggamma"), res[True], res[False]):
        assert torch.isfinite(a).all(), nm
        assert rel_inf(a, r) <= 1e-6, (nm, rel_inf(a, r))
