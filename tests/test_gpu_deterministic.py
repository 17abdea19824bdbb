"""Fixed-order reductions of the training reverse (grr_common.h, "Fixed-order reductions"): every
per-graph scalar, tap and multiM gradient is summed from per-contributor slots in a fixed order, so a
reverse run twice on the same inputs gives bitwise the same result (the float atomics of rounds 1-3
did not), and the destinations are accumulated into (dst += sum) as before.  The values themselves
are pinned by the gradient tests (test_gpu_grad.py, test_gpu_term_rows.py, ...)."""
import pytest
import torch

from tests.test_gpu_parity import DEV

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def irdu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import irdu_amd
    irdu_amd.load_native()
    return irdu_amd


@pytest.fixture(scope="module")
def K():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import irdu_amd
    irdu_amd.load_native()
    from irdu_amd import kernels
    yield kernels
    kernels.set_term_rows(True)


def _twice(fn):
    a = [t.clone() for t in fn()]
    torch.cuda.synchronize()
    b = [t.clone() for t in fn()]
    torch.cuda.synchronize()
    return a, b


def _equal(a, b, names):
    for name, x, y in zip(names, a, b):
        assert torch.isfinite(x).all(), name
        assert torch.equal(x, y), f"{name}: not bitwise reproducible (max diff {float((x - y).abs().max())})"


@pytest.mark.parametrize("rows", [True, False], ids=["rows", "pixels"])
@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("shape", [(2, 4, 3, 40, 256), (3, 2, 2, 17, 100), (1, 2, 3, 11, 300)],
                         ids=lambda s: "b{}g{}f{}h{}w{}".format(*s))
def test_term_reverse_reductions_bitwise(K, rows, mode, shape):
    b, G, F, h, w_ = shape
    torch.manual_seed(mode + 10 * h)
    C = G * F
    x = torch.randn(b, C, h, w_, device=DEV)
    g = torch.randn(b, C, h, w_, device=DEV)
    taps = torch.randn(C, 5, device=DEV) * 0.5
    w = torch.rand(b, G, 2 if mode == 1 else 4, h, w_, device=DEV)
    lg = torch.log(torch.linspace(0.05, 0.5, G, device=DEV)) if mode == 2 else None
    scale = torch.rand(G, device=DEV) + 0.5
    init = torch.randn(G, device=DEV)

    def run():
        K.set_term_rows(rows)
        gw = torch.zeros_like(w)
        gdot = init.clone()                       # accumulated into
        ggam = init.clone() if mode == 2 else torch.zeros(0, device=DEV)
        gtaps = torch.zeros_like(taps)
        v = K.bwd_term_fused(mode, x, g, taps, w, lg, scale, 0.7, gw, ggam if mode == 2 else None, gdot, gtaps, G)
        return v, gw, gdot, ggam, gtaps

    a, bb = _twice(run)
    _equal(a, bb, ["v", "gw", "gdot", "ggamma", "gtaps"])
    # dst += sum: the accumulated destination minus its initial value is the launch's own sum
    ref = run()
    gdot0 = torch.zeros(G, device=DEV)
    gw0, gt0 = torch.zeros_like(w), torch.zeros_like(taps)
    K.bwd_term_fused(mode, x, g, taps, w, lg, scale, 0.7, gw0, torch.zeros(G, device=DEV) if mode == 2 else None,
                     gdot0, gt0, G)
    torch.cuda.synchronize()
    assert torch.allclose(ref[2] - init, gdot0, rtol=1e-5, atol=1e-6 * float(gdot0.abs().max()))


@pytest.mark.parametrize("rows", [True, False], ids=["rows", "pixels"])
def test_edge_weights_reverse_bitwise(K, rows):
    torch.manual_seed(3)
    b, G, F, h, w_ = 2, 4, 3, 33, 136
    feat = torch.randn(b, G * F + 5, h, w_, device=DEV)
    multiM = torch.rand(G, F, device=DEV) + 0.5
    w = torch.softmax(torch.randn(b, G, 4, h, w_, device=DEV), dim=2)
    gw = torch.randn(b, G, 4, h, w_, device=DEV)

    def run():
        K.set_term_rows(rows)
        gfeat = torch.zeros_like(feat)
        gM = torch.zeros(G, F, device=DEV)
        K.bwd_edge_weights(feat, 2, G, F, multiM, w, gw, gfeat, gM)
        return gfeat, gM

    a, bb = _twice(run)
    _equal(a, bb, ["gfeat", "gmultiM"])


@pytest.mark.parametrize("width", [64, 131, 256], ids=["w64", "w131-pixels", "w256"])
def test_depthwise_and_gate_reverses_bitwise(K, width):
    torch.manual_seed(width)
    b, c, h = 2, 6, 24
    hh = torch.randn(b, c, h, width, device=DEV)
    g = torch.randn(b, c, h, width, device=DEV)
    wdw = torch.randn(c, 1, 3, 3, device=DEV)

    def run_dw():
        gwdw = torch.zeros_like(wdw)
        gh = K.dwconv3_bwd(g, hh, wdw, gwdw)
        return gh, gwdw

    a, bb = _twice(run_dw)
    _equal(a, bb, ["gh", "gwdw"])
    if width % 4 == 0 or width <= 64:
        gq = torch.randn(b, c // 2, h, width, device=DEV)
        scale = torch.tensor([0.7], device=DEV)

        def run_gate():
            gwdw = torch.zeros_like(wdw)
            gdot = torch.zeros(1, device=DEV)
            gh = K.lnb_gate_dw3_bwd(None, gq, scale, hh, wdw, gwdw, gdot)
            return gh, gwdw, gdot

        a, bb = _twice(run_gate)
        _equal(a, bb, ["gh", "gwdw", "gdot"])


def test_glue_reductions_bitwise(K):
    torch.manual_seed(5)
    b, G, F, h, w_ = 3, 4, 3, 20, 36
    u, v = torch.randn(b, G * F, h, w_, device=DEV), torch.randn(b, G * F, h, w_, device=DEV)

    def run_dot():
        out = torch.zeros(G, device=DEV)
        K.bwd_graph_dot(u, v, out, G, coef=0.3)
        return (out,)

    a, bb = _twice(run_dot)
    _equal(a, bb, ["gdot"])
    ref = (u.double() * v.double()).reshape(b, G, -1).sum(dim=(0, 2)) * 0.3
    assert torch.allclose(a[0].double(), ref, rtol=1e-5, atol=1e-5)


def test_msgf_training_gradients_bitwise(irdu):
    """A whole training reverse (every term reverse, edge weights, LNB blocks, side and level streams at
    their defaults) run twice: identical gradients."""
    import torch.nn.functional as F
    torch.manual_seed(11)
    m = irdu.MultiScaleGraphFilter(3, 3, ngraphs=8, n_cgd_iters=4).to(DEV)
    x = torch.rand(2, 3, 64, 96, device=DEV)
    t = torch.rand(2, 3, 64, 96, device=DEV)
    runs = []
    for _ in range(2):
        for p in m.parameters():
            p.grad = None
        F.mse_loss(m(x), t).backward()
        torch.cuda.synchronize()
        runs.append([p.grad.clone() for p in m.parameters()])
    for (name, _), a, b in zip(m.named_parameters(), *runs):
        assert torch.equal(a, b), name


def test_window_reverse_reductions_bitwise(K):
    """The window-graph reverse (taps, per-graph scalars, multiM) and the sub-API reverses are fixed-order
    too."""
    torch.manual_seed(9)
    b, G, fs, f, h, w_ = 2, 3, 3, 4, 21, 37
    delta = ((-1, 0), (0, -1), (0, 1), (1, 0), (-1, -1), (1, 1), (-2, 0), (0, 2))
    k = len(delta)
    s = torch.randn(b, G, fs, h, w_, device=DEV)
    bt = torch.randn_like(s)
    wt = torch.softmax(torch.randn(b, G, k, h, w_, device=DEV), dim=2)
    sc = torch.rand(G, device=DEV) + 0.5
    lg = torch.log(torch.full((G,), 0.05, device=DEV))
    feat = torch.randn(b, G * f, h, w_, device=DEV)
    M = torch.rand(G, f, device=DEV) + 0.5

    def run():
        gw = torch.zeros_like(wt)
        gdot, ggam, gt = torch.zeros(G, device=DEV), torch.zeros(G, device=DEV), torch.zeros(5, device=DEV)
        o, gs = K.win_bwd_gtv(s, bt, wt, delta, True, lg, sc, 0.7, gw, gdot, ggam, G)
        l, gs2 = K.win_bwd_glr(s, bt, wt, delta, sc, -1.0, gw, gdot, G)
        K.win_bwd_tapgrad(bt, o, K.WTAP_T, G, sc, gt)
        gfeat, gM = torch.zeros_like(feat), torch.zeros(G, f, device=DEV)
        K.win_bwd_edge_weights(feat, 0, G, f, M, wt, gw.clone(), delta, gfeat, gM)
        return o, gs, l, gs2, gw, gdot, ggam, gt, gfeat, gM

    a, bb = _twice(run)
    _equal(a, bb, ["o", "gs", "l", "gs2", "gw", "gdot", "ggamma", "gtaps", "gfeat", "gmultiM"])


def test_subapi_reverse_reductions_bitwise(K):
    torch.manual_seed(12)
    b, G, f, h, w_ = 2, 4, 3, 19, 23
    x5 = torch.randn(b, G, f, h, w_, device=DEV)
    g = torch.randn_like(x5)
    M = torch.rand(G, f, device=DEV) + 0.5
    p = [torch.rand(G * f, device=DEV) for _ in range(4)]      # p01, p02a, p02b, p03 per channel
    st = K.Stencil(*[t.data_ptr() for t in p])

    def run():
        gM = torch.zeros(G, f, device=DEV)
        gf = K.normalize_features_bwd(x5, M, g, gM)
        gt = torch.zeros(G * f, 5, device=DEV)
        gx = K.stats_conv_bwd(x5, st, False, g, gt)
        return gf, gM, gx, gt

    a, bb = _twice(run)
    _equal(a, bb, ["gf", "gmultiM", "gx", "gtaps"])
