"""grr_bwd_term_fused's row-streaming kernel (W <= 256; wider rows as column strips) against its per-pixel kernel, for the three
operator terms (GLR, pair Laplacian, prox) and every instantiated F: the v output, the weight
gradient (summed over the graph's channels through LDS), and the per-graph / per-channel
reductions (<a, z>, gamma, taps).  The per-pixel kernel is itself pinned by the gradient tests
(reference autograd golden + float64 oracle autograd, test_gpu_grad.py)."""
import pytest
import torch

from tests.test_gpu_parity import DEV, rel_err

pytestmark = pytest.mark.gpu

# W > 256: column strips of 248 owned columns (300: 2 strips, 512: 3, 744: 3 whole strips)
CASES = [(2, 4, 3, 20, 256), (1, 3, 1, 9, 32), (1, 2, 2, 17, 100), (1, 2, 4, 70, 200), (3, 2, 3, 2, 64),
         (1, 1, 3, 300, 128), (1, 2, 3, 11, 300), (1, 2, 4, 8, 512), (1, 1, 2, 6, 744)]


@pytest.fixture(scope="module")
def K():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import irdu_amd
    irdu_amd.load_native()
    from irdu_amd import kernels
    yield kernels
    kernels.set_term_rows(True)


def _run(K, mode, x, g, taps, w, lg, scale, G, rows):
    K.set_term_rows(rows)
    gw = torch.full_like(w, 0.5)           # accumulated into (+=)
    gdot = torch.zeros(G, device=DEV)
    ggam = torch.zeros(G, device=DEV) if mode == 2 else None
    gtaps = torch.zeros_like(taps)
    v = K.bwd_term_fused(mode, x, g, taps, w, lg, scale, 0.7, gw, ggam, gdot, gtaps, G)
    torch.cuda.synchronize()
    return v.cpu(), gw.cpu(), gdot.cpu(), None if ggam is None else ggam.cpu(), gtaps.cpu()


@pytest.mark.parametrize("case", CASES, ids=lambda c: "b{}g{}f{}h{}w{}".format(*c))
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_term_rows_equal_per_pixel(K, case, mode):
    b, G, F, h, w_ = case
    torch.manual_seed(mode * 100 + h + w_)
    C = G * F
    x = torch.randn(b, C, h, w_, device=DEV)
    g = torch.randn(b, C, h, w_, device=DEV)
    taps = torch.randn(C, 5, device=DEV) * 0.5
    planes = 2 if mode == 1 else 4
    w = torch.rand(b, G, planes, h, w_, device=DEV)
    lg = torch.log(torch.linspace(0.05, 0.5, G, device=DEV)) if mode == 2 else None
    scale = torch.rand(G, device=DEV) + 0.5
    ref = _run(K, mode, x, g, taps, w, lg, scale, G, rows=False)
    got = _run(K, mode, x, g, taps, w, lg, scale, G, rows=True)
    names = ["v", "gw", "gdot", "ggamma", "gtaps"]
    for name, a, r in zip(names, got, ref):
        if r is None:
            continue
        assert torch.isfinite(a).all(), name
        if name in ("v", "gw"):
            assert rel_err(a, r) <= 2e-6, (name, rel_err(a, r))
        else:
            # reductions of O(1) terms in two summation orders: fp32 error grows like sqrt(N) eps,
            # so a sum that cancels to far below sqrt(N) is held to that scale (a missing or doubled
            # column would still be off by O(rows x channels))
            n = b * F * h * w_
            scale = max(float(r.abs().max()), n ** 0.5)
            err = float((a.double() - r.double()).abs().max())
            assert err <= 2e-5 * scale, (name, err, scale)


WIDE_F = [(2, 2, 6, 18, 256), (1, 2, 12, 9, 256), (1, 2, 16, 7, 128), (2, 1, 12, 12, 64), (1, 1, 6, 5, 32),
          (1, 2, 6, 7, 512), (1, 1, 12, 5, 300)]


@pytest.mark.parametrize("case", WIDE_F, ids=lambda c: "b{}g{}f{}h{}w{}".format(*c))
def test_term_rows_large_f_equal_five_pass(K, case):
    """F > 4 (the v1.0 model's F = 6 and 12 levels): the row kernel against the five-pass reverse
    (stencils, Z-reverse, tap gradients, adjoint stencil) on all three terms, through solver_grad."""
    from irdu_amd import solver_grad as SG
    b, G, F, h, w_ = case
    torch.manual_seed(F * 10 + h)
    C = G * F
    # x at a scale where |C x| sits far from gamma (0.05..0.5) except on a set of measure ~0: the two
    # paths round s = P x differently in the last place, which could flip an edge's soft-threshold
    # branch if |C x| were within rounding of gamma
    x = 100.0 * torch.randn(b, C, h, w_, device=DEV)
    g = torch.randn(b, C, h, w_, device=DEV)
    taps = torch.randn(C, 5, device=DEV) * 0.5
    wl = torch.rand(b, G, 4, h, w_, device=DEV)
    cg = torch.rand(b, G, 2, h, w_, device=DEV)
    scale = torch.rand(G, device=DEV) + 0.5
    lg = torch.log(torch.linspace(0.05, 0.5, G, device=DEV))
    res = {}
    saved = SG.FUSED
    try:
        for fused in (False, True):
            SG.FUSED = fused
            outs = []
            for term in ("glr", "gtv", "prox"):
                out = torch.zeros_like(x)
                gw = torch.zeros_like(cg if term == "gtv" else wl)
                gs = torch.zeros(G, device=DEV)
                gt = torch.zeros_like(taps)
                if term == "glr":
                    SG.glr_term_bwd(x, g, taps, wl, scale, 0.7, G, out, gw, gs, gt)
                    outs.append((out, gw, gs, gt))
                elif term == "gtv":
                    SG.gtv_term_bwd(x, g, taps, cg, scale, 0.7, G, out, gw, gs, gt)
                    outs.append((out, gw, gs, gt))
                else:
                    assert SG._use_fused(x, G) == fused
                    st = tuple(taps[:, 0].contiguous() for _ in range(4))
                    lvl = SG._Level(wl, cg, wl, st, st, lg, torch.log(scale), lg, G)
                    lvl.tapsG = taps
                    lvl.prox_bwd(x, g, out)
                    outs.append((out, lvl.gwG, lvl.gro, lvl.ggam, lvl.gtapG))
            res[fused] = outs
    finally:
        SG.FUSED = saved
    torch.cuda.synchronize()
    for t, (a_set, r_set) in enumerate(zip(res[True], res[False])):
        for i, (a, r) in enumerate(zip(a_set, r_set)):
            assert torch.isfinite(a).all()
            assert rel_err(a.cpu(), r.cpu()) <= 2e-5, (t, i, rel_err(a.cpu(), r.cpu()))


EDGE_CASES = [(2, 4, 3, 20, 256), (1, 3, 1, 9, 32), (1, 2, 2, 17, 100), (1, 2, 6, 33, 200), (3, 2, 4, 2, 64),
              (1, 1, 3, 140, 128), (1, 2, 12, 9, 64),
              (1, 2, 6, 7, 512), (2, 1, 3, 5, 300), (1, 2, 4, 6, 744)]   # W > 256: column strips


@pytest.mark.parametrize("case", EDGE_CASES, ids=lambda c: "b{}g{}f{}h{}w{}".format(*c))
def test_edge_weights_reverse_rows_equal_per_pixel(K, case):
    """grr_bwd_edge_weights' row kernel (F in {1, 2, 3, 4, 6}; W > 256 in column strips; F = 12 falls back) against the
    per-pixel kernel, on a GTV/GLR slab at a channel offset of a wider feature tensor."""
    b, G, F, h, w_ = case
    torch.manual_seed(F * 7 + h)
    C = G * F
    feat = torch.randn(b, 2 * C, h, w_, device=DEV)
    feat[:, C:C + 1, :2, :3] = 0.0                      # some zero-norm pixels (the 1e-12 floor)
    multiM = torch.rand(G, F, device=DEV) + 0.5
    wts = K.edge_weights(feat, C, G, F, multiM)
    w = wts[0] if isinstance(wts, tuple) else wts
    gw = torch.randn_like(w)
    outs = []
    for rows in (False, True):
        K.set_term_rows(rows)
        gfeat = torch.zeros_like(feat)
        gM = torch.zeros_like(multiM)
        K.bwd_edge_weights(feat, C, G, F, multiM, w, gw, gfeat, gM)
        torch.cuda.synchronize()
        outs.append((gfeat.cpu(), gM.cpu()))
    K.set_term_rows(True)
    (rf, rm), (af, am) = outs
    assert torch.isfinite(af).all()
    assert rel_err(af, rf) <= 2e-6
    assert rel_err(am, rm) <= 2e-5
