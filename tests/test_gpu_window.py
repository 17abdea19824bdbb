"""GPU parity of the window-graph MixtureGTV path (window_ops.hip via irdu_amd.window_graph).

Against the reference's own outputs (tests/golden/window_*.npz, from REF7 =
lib/model_GLR_GTV_deep_v7.py) and, at larger / other shapes, against the CPU oracle
(oracle/window_oracle.py, pinned to the same fixtures).  Tolerance: 1e-4 relative
(max-abs error / max-abs reference), as the north_star states for fp32 outputs.
"""
import numpy as np
import pytest
import torch

from oracle import window_oracle as O
from tests.golden_io import load_golden

pytestmark = pytest.mark.gpu
RTOL = 1e-4
DEV = "cuda"
WINDOWS = ("ring3", "diamond5", "full5")


@pytest.fixture(scope="module")
def wg():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import irdu_amd
    irdu_amd.load_native()
    from irdu_amd import window_graph
    return window_graph


def rel_err(a, b):
    a = a.detach().double().cpu()
    b = torch.as_tensor(np.asarray(b) if not isinstance(b, torch.Tensor) else b).double().cpu()
    assert a.shape == b.shape, (a.shape, b.shape)
    return float((a - b).abs().max()) / max(float(b.abs().max()), 1e-30)


def _ops_params(d, name, pre):
    full = f"{name}/p/{pre}"
    return {k[len(full):]: torch.from_numpy(d[k].copy()) for k in d.files if k.startswith(full)}


def _window(name):
    return {"ring3": np.array([1, 1, 1, 1, 0, 1, 1, 1, 1]).reshape(3, 3),
            "diamond5": np.array([0, 0, 1, 0, 0, 0, 1, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 1, 0, 0, 0, 1, 0, 0])
            .reshape(5, 5),
            "full5": np.array([1] * 12 + [0] + [1] * 12).reshape(5, 5)}[name]


@pytest.mark.parametrize("name", WINDOWS)
def test_window_modules_vs_reference_golden(wg, name):
    d = load_golden("window_ops_v7.npz")
    feat = torch.from_numpy(d[f"{name}/feat"]).to(DEV)
    x = torch.from_numpy(d[f"{name}/x"]).to(DEV)
    b, g, f, h, w = feat.shape
    glr = wg.GLRFast(3, f, g, _window(name)).to(DEV)
    gtv = wg.GTVFast(3, f, g, _window(name)).to(DEV)
    glr.load_state_dict(_ops_params(d, name, "glr."))
    gtv.load_state_dict(_ops_params(d, name, "gtv."))
    with torch.no_grad():
        wl, deg = glr.extract_edge_weights(feat)
        wgt, _ = gtv.extract_edge_weights(feat)
        assert rel_err(wl, d[f"{name}/wL"]) <= 1e-5
        assert rel_err(wgt, d[f"{name}/wG"]) <= 1e-5
        assert rel_err(deg, d[f"{name}/degL"]) <= 1e-5
        wl_ref = torch.from_numpy(d[f"{name}/wL"]).to(DEV)
        wg_ref = torch.from_numpy(d[f"{name}/wG"]).to(DEV)
        assert rel_err(glr(x, wl_ref), d[f"{name}/glr"]) <= RTOL
        assert rel_err(gtv(x, wg_ref), d[f"{name}/gtv"]) <= RTOL


def _load_mixture(wg, g):
    m = wg.MixtureGTV(3, 4, 3, 8, wg.CONNECTION_FLAGS_5x5_small, 4, 0.5, 0.1, torch.tensor([[0.1]]),
                      torch.tensor([[0.1]]), torch.tensor([[0.001]]))
    m.load_state_dict({k[2:]: torch.from_numpy(g[k].copy()) for k in g.files if k.startswith("p/")})
    return m.to(DEV).eval()


def test_window_mixture_vs_reference_golden(wg):
    g = load_golden("window_v7.npz")
    m = _load_mixture(wg, g)
    with torch.no_grad():
        out = m(torch.from_numpy(g["in/noisy"]).to(DEV))
    assert rel_err(out, g["out/y"]) <= RTOL


def test_window_solver_vs_reference_features(wg):
    """The solver alone, fed the reference's own features and dc term (isolates the HIP
    solver from the stock-PyTorch feature CNN)."""
    g = load_golden("window_v7.npz")
    m = _load_mixture(wg, g)
    p = {k[2:]: torch.from_numpy(g[k].copy()) for k in g.files if k.startswith("p/")}
    feats = torch.from_numpy(g["out/feats"])
    y = torch.from_numpy(g["in/noisy"]) - torch.from_numpy(g["out/dc"])
    ref = O.mixture_solve(y, feats[:, :-12], p, 4, 3, O.window_edges(wg.CONNECTION_FLAGS_5x5_small))
    with torch.no_grad():
        got = m.solve(y.to(DEV).contiguous(), feats[:, :-12].contiguous().to(DEV), feats.to(DEV).contiguous())
    assert rel_err(got, ref) <= RTOL


@pytest.mark.parametrize("name,shape,iters", [("ring3", (2, 5, 3, 40, 70), 6), ("diamond5", (1, 6, 3, 48, 136), 4),
                                              ("full5", (2, 3, 12, 33, 65), 6), ("diamond5", (1, 2, 3, 16, 300), 5)])
def test_window_solver_vs_oracle_random(wg, name, shape, iters):
    """Odd sizes, several tiles in both directions, ragged last tiles, F=12 features, 6 stages."""
    b, g, f, h, w = shape
    gen = torch.Generator().manual_seed(2207 + h)
    cw = _window(name)
    delta = O.window_edges(cw)
    p = {"GTVmodule00.multiM": 0.5 + torch.rand((g, f), generator=gen),
         "GLRmodule00.multiM": 0.5 + torch.rand((g, f), generator=gen),
         "ro00": 0.1 + 0.5 * torch.rand(g, generator=gen), "muys00": 0.1 + 0.5 * torch.rand(g, generator=gen),
         "gamma00": torch.log(0.002 + 0.01 * torch.rand(g, generator=gen)),
         "alphaCGD": 0.2 + 0.6 * torch.rand((iters, g), generator=gen),
         "betaCGD": 0.05 + 0.35 * torch.rand((iters, g), generator=gen)}
    for pre in ("GTVmodule00.", "GLRmodule00."):
        for k, lo, span in (("p01", 0.8, 0.4), ("p02a", 0.2, 0.6), ("p02b", 0.2, 0.6), ("p03", 0.1, 0.5)):
            p[pre + "stats_kernel_" + k] = lo + span * torch.rand(1, generator=gen)
    y = torch.rand((b, 3, h, w), generator=gen)
    feats = torch.randn((b, g * f, h, w), generator=gen)
    ref = O.mixture_solve(y, feats, p, g, f, delta, n_cgd_iters=iters)
    m = wg.MixtureGTV.__new__(wg.MixtureGTV)
    torch.nn.Module.__init__(m)
    m.n_graphs, m.n_node_fts, m.n_cgd_iters = g, f, iters
    m.GTVmodule00 = wg.GTVFast(3, f, g, cw)
    m.GLRmodule00 = wg.GLRFast(3, f, g, cw)
    m.ro00, m.muys00, m.gamma00 = (torch.nn.Parameter(p[k]) for k in ("ro00", "muys00", "gamma00"))
    m.alphaCGD, m.betaCGD = torch.nn.Parameter(p["alphaCGD"]), torch.nn.Parameter(p["betaCGD"])
    for pre, mod in (("GTVmodule00.", m.GTVmodule00), ("GLRmodule00.", m.GLRmodule00)):
        mod.load_state_dict({k[len(pre):]: v for k, v in p.items() if k.startswith(pre)})
    m = m.to(DEV)
    with torch.no_grad():
        got = m.solve(y.to(DEV), feats.to(DEV))
    assert rel_err(got, ref) <= RTOL


def test_window_sequence_denoiser_small(wg):
    """MultiScaleSequenceDenoiser (REF7:1019-1087: 24 graphs, n_cnn_fts 128, K=12) end to end vs
    the oracle on one 32x48 patch, solver scalars moved off their init."""
    torch.manual_seed(2207)
    model = wg.MultiScaleSequenceDenoiser()
    mix = model.mixtureGLR_block03
    with torch.no_grad():
        mix.muys00.fill_(0.4); mix.ro00.fill_(0.3); mix.gamma00.fill_(float(np.log(0.005)))
    p = {k: v.detach().clone() for k, v in model.state_dict().items()}
    img = torch.rand((1, 3, 32, 48))
    ref = O.sequence_denoiser_v7(img, p)
    model = model.to(DEV).eval()
    with torch.no_grad():
        out = model(img.to(DEV))
    assert rel_err(out, ref) <= RTOL


V1_WINDOWS = {"ring3": (2, 3, np.array([1, 1, 1, 1, 0, 1, 1, 1, 1]).reshape(3, 3)),
              "full5": (2, 2, np.array([1] * 12 + [0] + [1] * 12).reshape(5, 5))}


@pytest.mark.parametrize("name", sorted(V1_WINDOWS))
def test_window_v1_block_vs_reference_golden(wg, name):
    from irdu_amd import window_graph_v1 as W1
    d = load_golden("window_v1.npz")
    g, f, cw = V1_WINDOWS[name]
    m = W1.MixtureGTV(3, g, f, cw, 6, 0.5, 0.1, torch.tensor([[0.1]]), torch.tensor([[0.1]]), torch.tensor([[0.001]]))
    pre = f"{name}/p/"
    m.load_state_dict({k[len(pre):]: torch.from_numpy(d[k].copy()) for k in d.files if k.startswith(pre)})
    m = m.to(DEV).eval()
    with torch.no_grad():
        out = m(torch.from_numpy(d[f"{name}/in"]).to(DEV))
    assert rel_err(out, d[f"{name}/out"]) <= RTOL


def test_window_v1_sequence_denoiser_vs_oracle(wg):
    """REF1 MultiScaleSequenceDenoiser (three blocks: K=8, K=8, K=24; 6 CG stages) end to end."""
    from irdu_amd import window_graph_v1 as W1
    torch.manual_seed(2201)
    model = W1.MultiScaleSequenceDenoiser()
    with torch.no_grad():
        for i in (1, 2, 3):
            mix = getattr(model, f"mixtureGLR_block0{i}")
            mix.muys00.fill_(0.3); mix.ro00.fill_(0.2); mix.gamma00.fill_(float(np.log(0.005)))
    p = {k: v.detach().clone() for k, v in model.state_dict().items()}
    img = torch.rand((2, 3, 32, 40))
    ref = O.sequence_denoiser_v1(img, p)
    model = model.to(DEV).eval()
    with torch.no_grad():
        out = model(img.to(DEV))
    assert rel_err(out, ref) <= RTOL


@pytest.mark.parametrize("name", WINDOWS)
def test_window_pair_weights_and_pair_solver(wg, name):
    """grr_win_pair_weights against a torch restatement of c_e(q) = w_e(q)^2 + [q + d_e inside]
    w_e'(q + d_e)^2, and the solver's pair-weight modes (CG step, first rhs, module apply)
    against the raw-weight modes they replace (same linear term, different summation order)."""
    from irdu_amd import kernels as K
    torch.manual_seed(31)
    b, g, fs, h, w = 2, 3, 3, 37, 70
    delta = O.window_edges(_window(name))
    k = len(delta)
    wgt = torch.softmax(torch.randn(b, g, k, h, w, device=DEV), 2)
    c = K.win_pair_weights(wgt, delta)
    ref = wgt.double() ** 2
    for e, (dy, dx) in enumerate(delta):
        o = [i for i, d in enumerate(delta) if tuple(d) == (-dy, -dx)][0]
        sh = torch.zeros_like(ref[:, :, e])
        ys, xs = slice(max(0, -dy), h - max(0, dy)), slice(max(0, -dx), w - max(0, dx))
        yd, xd = slice(max(0, dy), h - max(0, -dy)), slice(max(0, dx), w - max(0, -dx))
        sh[:, :, ys, xs] = wgt.double()[:, :, o, yd, xd] ** 2
        ref[:, :, e] += sh
    assert rel_err(c, ref) <= 1e-6
    x = torch.randn(b, g, fs, h, w, device=DEV)
    y = torch.randn(b, g, fs, h, w, device=DEV)
    y1 = torch.randn(b, fs, h, w, device=DEV)
    wl = torch.softmax(torch.randn(b, g, k, h, w, device=DEV), 2)
    taps = torch.tensor([1.3, -0.2, -0.15, -0.25, -0.1], device=DEV)
    ro, mu = torch.rand(g, device=DEV) + 0.2, torch.rand(g, device=DEV) + 0.2
    alpha, beta = torch.rand(g, device=DEV), torch.rand(g, device=DEV)
    u0 = torch.randn_like(x)
    raw0 = K.win_solver(0, x, y, wgt, taps, ro, delta, g, fs, wL=wl, tapsL=taps, mu=mu, alpha=alpha, beta=beta,
                        u_prev=u0)
    got0 = K.win_solver(0, x, y, c, taps, ro, delta, g, fs, wL=wl, tapsL=taps, mu=mu, alpha=alpha, beta=beta,
                        u_prev=u0, pair=True)
    assert rel_err(got0[0], raw0[0]) <= 1e-5 and rel_err(got0[1], raw0[1]) <= 1e-5
    raw1, _ = K.win_solver(1, x, y1, wgt, taps, ro, delta, g, fs)
    got1, _ = K.win_solver(1, x, y1, c, taps, ro, delta, g, fs, pair=True)
    assert rel_err(got1, raw1) <= 1e-5
    with pytest.raises(ValueError):
        K.win_solver(2, x, y1, c, taps, ro, delta, g, fs, log_gamma=torch.zeros(g, device=DEV), pair=True)
