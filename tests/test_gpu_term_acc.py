"""Fused reverse passes against the unfused ones they replace.

grr_bwd_term_fused_acc (the row-streaming term reverse with the x-gradient pass P*(v) inside) against
grr_bwd_term_fused + grr_bwd_stencil mode 3 on the same inputs, for the three operator terms: the
accumulated x-gradient, the weight gradient and the per-graph / per-channel reductions.  Shapes cover
one- and two-column lanes (W <= 128, where the fused pass runs), row segments with a ragged last segment
(the segment's halo rows), the image's first and last rows, F up to 16.  The two-pass path
is itself pinned by test_gpu_term_rows.py and the gradient tests.  grr_bwd_cg_glue with the half level's
x-gradient folded in (gx_half) against grr_bwd_unpool2_acc + the plain glue."""
import pytest
import torch

from tests.test_gpu_parity import DEV, rel_err

pytestmark = pytest.mark.gpu

# (B, G, F, H, W): H = 70 / 100 / 300 split into row segments (32 rows) with a ragged last one; W = 256 / 512
# check that the fused pass declines them
CASES = [(2, 4, 3, 64, 64), (1, 3, 3, 70, 128), (2, 2, 6, 100, 100), (1, 2, 3, 300, 128), (3, 2, 3, 2, 64),
         (1, 1, 12, 40, 128), (1, 2, 4, 9, 32), (1, 1, 1, 1, 64), (2, 1, 16, 33, 96), (1, 2, 6, 37, 512),
         (1, 2, 3, 20, 256)]


@pytest.fixture(scope="module")
def K():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import irdu_amd
    irdu_amd.load_native()
    from irdu_amd import kernels
    kernels.set_term_acc_max_w(1 << 20)   # the ring kernel's pass at every width (default: W <= 128)
    yield kernels
    kernels.set_term_acc_max_w(128)
    kernels.set_term_rows(True)


# level 1: the register-prefetch row kernel (one strip of <= 2-column lanes); level 2 (default): the
# LDS-ring kernel wherever it applies (gx rows in its slots: every width, strips included), else level 1
LEVELS = [1, 2]


def _inputs(mode, case):
    b, G, F, h, w_ = case
    torch.manual_seed(mode * 1000 + h * 7 + w_)
    C = G * F
    x = torch.randn(b, C, h, w_, device=DEV)
    g = torch.randn(b, C, h, w_, device=DEV)
    taps = torch.randn(C, 5, device=DEV) * 0.5
    w = torch.rand(b, G, 2 if mode == 1 else 4, h, w_, device=DEV)
    lg = torch.log(torch.linspace(0.05, 0.5, G, device=DEV)) if mode == 2 else None
    scale = torch.rand(G, device=DEV) + 0.5
    gx0 = torch.randn(b, C, h, w_, device=DEV)
    return x, g, taps, w, lg, scale, gx0


def _bufs(mode, w, taps, G):
    return (torch.full_like(w, 0.5), torch.zeros(G, device=DEV) if mode == 2 else None,
            torch.zeros(G, device=DEV), torch.zeros_like(taps))


@pytest.mark.parametrize("case", CASES, ids=lambda c: "b{}g{}f{}h{}w{}".format(*c))
@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("level", LEVELS)
def test_term_acc_equals_two_pass(K, case, mode, level):
    b, G, F, h, w_ = case
    K.set_term_rows(level)
    x, g, taps, w, lg, scale, gx0 = _inputs(mode, case)
    if not K.term_acc_ok(mode, x, G, g, gx0):
        # register kernel: W > 128 (4-column lanes, strips) stays on the two-pass path
        assert level == 1 and w_ > 128, (mode, case)
        return
    gw_r, gg_r, gd_r, gt_r = _bufs(mode, w, taps, G)
    v = K.bwd_term_fused(mode, x, g, taps, w, lg, scale, 0.7, gw_r, gg_r, gd_r, gt_r, G)
    gx_r = gx0.clone()
    K.bwd_stencil(v, taps, K.ST_P_ADJ, G, scale, out=gx_r)
    gw_a, gg_a, gd_a, gt_a = _bufs(mode, w, taps, G)
    gx_a = gx0.clone()
    K.bwd_term_fused_acc(mode, x, g, taps, w, lg, scale, 0.7, gx_a, gw_a, gg_a, gd_a, gt_a, G)
    torch.cuda.synchronize()
    # gx: the same expression in the same order as the stencil pass; the rest: the same kernel arithmetic
    assert rel_err(gx_a.cpu(), gx_r.cpu()) <= 1e-6, rel_err(gx_a.cpu(), gx_r.cpu())
    assert rel_err(gw_a.cpu(), gw_r.cpu()) <= 1e-6
    for name, a, r in (("gdot", gd_a, gd_r), ("ggamma", gg_a, gg_r), ("gtaps", gt_a, gt_r)):
        if r is None:
            continue
        err = float((a.double() - r.double()).abs().max())
        assert err <= 1e-5 * max(float(r.abs().max()), 1.0), (name, err)


@pytest.mark.parametrize("level,case", [(1, (2, 4, 3, 70, 128)), (2, (2, 4, 3, 70, 128)), (2, (1, 2, 6, 40, 512)),
                                        (2, (2, 4, 3, 33, 256))])
def test_glr_then_pair_equals_padj2(K, level, case):
    """Two accumulating calls on one gx (GLR, then pair: the level's terms_bwd) equal the padj2 sweep."""
    K.set_term_rows(level)
    b, G, F, h, w_ = case
    x, g, taps0, w0, _, s0, gx0 = _inputs(0, case)
    _, _, taps1, w1, _, s1, _ = _inputs(1, case)
    gx_r, gx_a = gx0.clone(), gx0.clone()
    b0, b1 = _bufs(0, w0, taps0, G), _bufs(1, w1, taps1, G)
    v0 = K.bwd_term_fused(0, x, g, taps0, w0, None, s0, -1.0, *b0, G)
    v1 = K.bwd_term_fused(1, x, g, taps1, w1, None, s1, -1.0, *b1, G)
    K.bwd_padj2(v0, taps0, s0, v1, taps1, s1, gx_r, G)
    b0, b1 = _bufs(0, w0, taps0, G), _bufs(1, w1, taps1, G)
    K.bwd_term_fused_acc(0, x, g, taps0, w0, None, s0, -1.0, gx_a, *b0, G)
    K.bwd_term_fused_acc(1, x, g, taps1, w1, None, s1, -1.0, gx_a, *b1, G)
    torch.cuda.synchronize()
    assert rel_err(gx_a.cpu(), gx_r.cpu()) <= 1e-6


@pytest.mark.parametrize("level", LEVELS)
def test_training_gradients_with_and_without_acc(K, level):
    """msgf's mixture reverse with the fused x-gradient passes against the two-pass path."""
    K.set_term_rows(level)
    import irdu_amd
    from irdu_amd import solver_grad as SG
    from tests.test_gpu_parity import perturb_mixture
    torch.manual_seed(5)
    m = irdu_amd.MultiScaleGraphFilter(3, 3, ngraphs=8, n_cgd_iters=4)
    perturb_mixture(m.localfilter, 9)
    m = m.to(DEV)
    y = torch.rand(2, 3, 64, 64, device=DEV)

    def grads(acc):
        SG.TERM_ACC = acc
        try:
            m.zero_grad(set_to_none=True)
            m(y).square().mean().backward()
            return {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}
        finally:
            SG.TERM_ACC = True

    ref, got = grads(False), grads(True)
    assert ref.keys() == got.keys()
    # the x-gradient passes agree to fp32 rounding (test_term_acc_equals_two_pass: 1e-6); through four
    # stages, the feature CNN's reverse and image-wide sums that cancel (a skip weight's gradient: 3.5 from
    # terms far larger) that rounding reaches a few 1e-5 of the largest gradient entry
    for k in ref:
        assert rel_err(got[k].cpu(), ref[k].cpu()) <= 2e-4, (k, rel_err(got[k].cpu(), ref[k].cpu()))


@pytest.mark.parametrize("shape", [(2, 6, 8, 12), (1, 3, 6, 10), (2, 12, 32, 64)], ids=str)
def test_cg_glue_with_half_level_equals_unpool_then_glue(K, shape):
    """grr_bwd_cg_glue's gx_half (U of the half level's x-gradient folded into the glue pass) against
    grr_bwd_unpool2_acc followed by the plain glue; W % 4 != 0 takes the scalar path."""
    b, c, h, w = shape
    G = 3
    torch.manual_seed(h * w)
    t = lambda *s: torch.randn(*s, device=DEV)  # noqa: E731
    gx, u, gun, up, gbb = (t(b, c, h, w) for _ in range(5))
    gxh = t(b, c, h // 2, w // 2)
    alpha, beta = torch.rand(G, device=DEV), torch.rand(G, device=DEV)

    def run(fold):
        ga, gb, bb = torch.zeros(G, device=DEV), torch.zeros(G, device=DEV), gbb.clone()
        x = gx.clone()
        if not fold:
            K.bwd_unpool2_acc(gxh, x)
        gu, gxo = K.bwd_cg_glue(x, u, gun, up, alpha, beta, bb, ga, gb, G, gx_half=gxh if fold else None)
        torch.cuda.synchronize()
        return [v.cpu() for v in (gu, gxo, bb, ga, gb)]

    for a, r in zip(run(True), run(False)):
        assert torch.equal(a, r) or rel_err(a, r) <= 1e-6, rel_err(a, r)


@pytest.mark.parametrize("shape", [(2, 6, 8, 12), (2, 12, 32, 64)], ids=str)
def test_cg_glue_with_padj_equals_padj2_then_glue(K, shape):
    """grr_bwd_cg_glue with the previous stage's padj2 sweep folded in (v1 / v2) and the half level's U
    against grr_bwd_padj2 + grr_bwd_unpool2_acc + the plain glue: the same operations in the same order."""
    b, c, h, w = shape
    G = 3
    torch.manual_seed(h + w)
    t = lambda *s: torch.randn(*s, device=DEV)  # noqa: E731
    gx, u, gun, up, gbb, v1, v2 = (t(b, c, h, w) for _ in range(7))
    gxh = t(b, c, h // 2, w // 2)
    t1, t2 = t(c, 5), t(c, 5)
    s1, s2 = torch.rand(G, device=DEV) + 0.5, torch.rand(G, device=DEV) + 0.5
    alpha, beta = torch.rand(G, device=DEV), torch.rand(G, device=DEV)

    def run(fold):
        ga, gb, bb = torch.zeros(G, device=DEV), torch.zeros(G, device=DEV), gbb.clone()
        x = gx.clone()
        if not fold:
            K.bwd_padj2(v1, t1, s1, v2, t2, s2, x, G)
            K.bwd_unpool2_acc(gxh, x)
        gu, gxo = K.bwd_cg_glue(x, u, gun, up, alpha, beta, bb, ga, gb, G, gx_half=gxh if fold else None,
                                padj=(v1, t1, s1, v2, t2, s2) if fold else None)
        torch.cuda.synchronize()
        return [v.cpu() for v in (gu, gxo, bb, ga, gb)]

    # the same operations in the same order; the compiler may contract the scale multiply into a different
    # fma in the two kernels (one rounding), which the per-graph sums (alpha, beta) carry at fp32 level
    n = b * (c // G) * h * w
    for name, a, r in zip(("gu", "gx", "gbb", "galpha", "gbeta"), run(True), run(False)):
        if name in ("galpha", "gbeta"):
            err = float((a.double() - r.double()).abs().max())
            assert err <= 2e-6 * max(float(r.abs().max()), n ** 0.5), (name, err)
        else:
            assert rel_err(a, r) <= 1e-6, (name, rel_err(a, r))


def test_training_gradients_with_and_without_unpool_glue(K):
    """msgf's mixture reverse with the previous stage's padj2 sweep and the half level's U folded into the
    next glue pass against the separate passes: the same arithmetic, so the same gradients."""
    import irdu_amd
    from irdu_amd import solver_grad as SG
    from tests.test_gpu_parity import perturb_mixture
    torch.manual_seed(6)
    m = irdu_amd.MultiScaleGraphFilter(3, 3, ngraphs=8, n_cgd_iters=5)
    perturb_mixture(m.localfilter, 11)
    m = m.to(DEV)
    y = torch.rand(2, 3, 96, 256, device=DEV)   # W = 256: the full level takes the padj2 sweep

    def grads(unpool, padj):
        SG.UNPOOL_GLUE, SG.PADJ_GLUE = unpool, padj
        try:
            m.zero_grad(set_to_none=True)
            m(y).square().mean().backward()
            return {k: p.grad.detach().cpu() for k, p in m.named_parameters() if p.grad is not None}
        finally:
            SG.UNPOOL_GLUE, SG.PADJ_GLUE = True, True

    ref = grads(False, False)
    for flags, tol in (((True, False), 1e-6), ((True, True), 1e-4)):
        # U folded in: the same arithmetic.  padj2 folded in: the same operations, one fma contraction may
        # differ (see above), carried through the reverse and image-wide sums that cancel
        got = grads(*flags)
        for k in ref:
            assert torch.equal(got[k], ref[k]) or rel_err(got[k], ref[k]) <= tol, (flags, k, rel_err(got[k], ref[k]))


@pytest.mark.parametrize("shape", [(2, 5, 8, 12), (3, 4, 6, 10), (16, 96, 64, 128), (1, 1, 2, 4), (2, 3, 256, 256)],
                         ids=str)
def test_pool2_equals_oracle_mean(K, shape):
    """grr_pool2 (the D the reverse applies to each stage's iterate and gradient) against the oracle's D in
    float64."""
    from oracle import graph_oracle as O
    torch.manual_seed(sum(shape))
    x = torch.randn(*shape)
    got = K.pool2(x.to(DEV)).cpu()
    want = O.pool2(x.double())
    assert got.shape == want.shape
    assert rel_err(got, want) <= 1e-6


@pytest.mark.parametrize("shape", [(2, 48, 16, 20), (1, 96, 33, 7)], ids=str)
def test_lnb_norm_bwd_skip_equals_separate_passes(K, shape):
    """grr_lnb_norm_bwd_skip (the LocalNonLinearBlock reverse's tail: s0 gout + the norm's data gradient,
    <gout, x>, the norm's weight gradient in one pass over gout) against lincomb + norm_bwd + graph_dot."""
    b, c, h, w = shape
    torch.manual_seed(c + h)
    x = torch.randn(b, c, h, w, device=DEV) + 0.3
    lnw = torch.rand(c, device=DEV) + 0.5
    gn, gout = torch.randn_like(x), torch.randn_like(x)
    skip = torch.tensor([0.7, 1.3], device=DEV)
    _, isd = K.lnb_norm(x, lnw)
    gl_a, gs_a = torch.zeros_like(lnw), torch.zeros(1, device=DEV)
    gx_a = K.lnb_norm_bwd_skip(x, lnw, isd, gn, gout, skip, gl_a, gs_a)
    gl_r, gs_r = torch.zeros_like(lnw), torch.zeros(1, device=DEV)
    gx_r = K.bwd_lincomb(gout, skip[0:1].contiguous(), None, None, 1)
    K.lnb_norm_bwd(x, lnw, isd, gn, gx_r, gl_r)
    K.bwd_graph_dot(gout, x, gs_r, 1)
    torch.cuda.synchronize()
    assert rel_err(gx_a, gx_r) <= 1e-6
    assert torch.equal(gl_a.cpu(), gl_r.cpu())
    n = x.numel()
    assert float((gs_a.double() - gs_r.double()).abs().max()) <= 2e-6 * max(float(gs_r.abs().max()), n ** 0.5)


def test_abstract_gradients_with_and_without_ln_skip(K):
    """The v1.0 model's training gradients with the LNB skip term inside the norm's reverse pass against
    the separate passes."""
    import irdu_amd
    from irdu_amd import solver_grad as SG
    torch.manual_seed(3)
    m = irdu_amd.AbtractMultiScaleGraphFilter(
        3, 3, dims=[8, 16, 16, 32], hidden_dims=[16, 32, 32, 64], nsubnets=[1, 1, 1, 1], ngraphs=[2, 4, 4, 8],
        num_blocks=[1, 1, 1, 1], num_blocks_out=1, n_cgd_iters=2).to(DEV)
    y = torch.rand(2, 3, 64, 64, device=DEV)

    def grads(fused):
        SG.LN_SKIP_FUSED = fused
        try:
            m.zero_grad(set_to_none=True)
            m(y).square().mean().backward()
            return {k: p.grad.detach().cpu() for k, p in m.named_parameters() if p.grad is not None}
        finally:
            SG.LN_SKIP_FUSED = True

    ref, got = grads(False), grads(True)
    assert ref.keys() == got.keys()
    for k in ref:
        assert rel_err(got[k], ref[k]) <= 1e-4, (k, rel_err(got[k], ref[k]))


@pytest.mark.parametrize("shape", [(2, 6, 8, 12), (2, 12, 32, 64), (1, 3, 2, 4), (2, 6, 6, 20)], ids=str)
@pytest.mark.parametrize("fold", [False, True])
def test_cg_glue_pool_equals_glue_then_pool2(K, shape, fold):
    """grr_bwd_cg_glue_pool (D gu written by the glue pass, row pairs per thread) against the plain glue
    followed by grr_pool2 of gu; with and without the previous stage's padj2 / U passes folded in.  The
    element-wise outputs are the same expressions; the per-graph sums run in another order."""
    b, c, h, w = shape
    G = 3
    torch.manual_seed(h * w + int(fold))
    t = lambda *s: torch.randn(*s, device=DEV)  # noqa: E731
    gx, u, gun, up, gbb, v1, v2 = (t(b, c, h, w) for _ in range(7))
    gxh = t(b, c, h // 2, w // 2)
    t1, t2 = t(c, 5), t(c, 5)
    s1, s2 = torch.rand(G, device=DEV) + 0.5, torch.rand(G, device=DEV) + 0.5
    alpha, beta = torch.rand(G, device=DEV), torch.rand(G, device=DEV)
    assert K.glue_pool_ok(gx)

    def run(pool):
        ga, gb, bb = torch.zeros(G, device=DEV), torch.zeros(G, device=DEV), gbb.clone()
        x = gx.clone()
        r = K.bwd_cg_glue(x, u, gun, up, alpha, beta, bb, ga, gb, G, gx_half=gxh if fold else None,
                          padj=(v1, t1, s1, v2, t2, s2) if fold else None, want_pool=pool)
        gu, gxo = r[:2]
        gud = r[2] if pool else K.pool2(gu)
        torch.cuda.synchronize()
        return [v.cpu() for v in (gu, gxo, gud, bb, ga, gb)]

    n = b * (c // G) * h * w
    for name, a, r in zip(("gu", "gx", "gud", "gbb", "galpha", "gbeta"), run(True), run(False)):
        if name in ("galpha", "gbeta"):
            err = float((a.double() - r.double()).abs().max())
            assert err <= 2e-6 * max(float(r.abs().max()), n ** 0.5), (name, err)
        else:
            assert rel_err(a, r) <= 1e-6, (name, rel_err(a, r))


def test_cg_glue_pool_rejects_odd_shapes(K):
    from irdu_amd._native import GrrError
    G = 3
    x = torch.randn(1, 6, 5, 8, device=DEV)      # odd H
    a = torch.rand(G, device=DEV)
    assert not K.glue_pool_ok(x)
    with pytest.raises(GrrError):
        K.bwd_cg_glue(x, x.clone(), None, None, a, None, None, torch.zeros(G, device=DEV), None, G, want_pool=True)
