"""grr_system_step2 (two CG stages per pass, temporal blocking, both half levels inside) against the
one-stage-per-launch sequence grr_system_half -> grr_system_step -> grr_system_half -> grr_system_step
and against the CPU oracle.

The fused kernel computes the same values with the same per-row arithmetic; the tolerance
below (2e-6 relative to the largest output) covers fp32 contraction differences between the
two code paths.  Shapes cover one row segment per (b, graph) (B*G >= 512 workgroups) and the
segmented grid of small batches (64-row segments, the stage-A lead of 9 rows crossing the
segment boundary), the top / bottom replicate clamps of the in-kernel rings at short H, F > 3 as
channel groups, the first pair (no u_prev / beta_a) and the last pair (skip, no u / D x outputs).
Widths other than 256 run the column-strip instance (256-lane windows, 16-column halo): W > 256 in
2-4 strips (the reference's 336 x 496 evaluation pad among them), narrower W % 8 == 0 as one strip
with lanes past the image edge.
"""
import pytest
import torch

from oracle import graph_oracle as O
from tests.test_gpu_parity import DEV, perturb_mixture, rel_err, sd_cpu

pytestmark = pytest.mark.gpu
TIGHT = 2e-6


@pytest.fixture(scope="module")
def irdu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import irdu_amd
    irdu_amd.load_native()
    return irdu_amd


def _setup(irdu, B, G, F, H, seed, W=256):
    from irdu_amd import kernels as K
    torch.manual_seed(seed)
    mix = irdu.MixtureGTVGLR(G, F, 0.5, 0.1, [[1e-3], [1e-4]], [[1e-4], [1e-4]], [[1e-4], [1e-4]], n_cgd_iters=4)
    perturb_mixture(mix, seed)
    with torch.no_grad():   # scales large enough that both levels matter
        mix.muys00.fill_(-1.0)
        mix.ro00.fill_(-1.5)
        mix.muys01.fill_(-1.2)
        mix.ro01.fill_(-1.6)
    mix = mix.to(DEV)
    f0 = torch.randn(B, 2 * G * F, H, W, device=DEV)
    f1 = torch.randn(B, 2 * G * F, H // 2, W // 2, device=DEV)
    _, cG0, wL0 = K.edge_weights_block(f0, G, F, mix.GTVmodule00.multiM, mix.GLRmodule00.multiM)
    _, cG1, wL1 = K.edge_weights_block(f1, G, F, mix.GTVmodule01.multiM, mix.GLRmodule01.multiM)
    C = G * F
    x = torch.rand(B, C, H, W, device=DEV)
    b = x + 0.1 * torch.randn(B, C, H, W, device=DEV)
    u = 0.05 * torch.randn(B, C, H, W, device=DEV)
    return mix, x, b, u, (wL0, cG0, wL1, cG1)


def _two_steps(irdu, mix, x, b, u, w, k, g, skip=None, y_skip=None, last=False):
    from irdu_amd import ops as OPS
    wL0, cG0, wL1, cG1 = w
    m = mix
    alpha, beta = m.alphaCGD, m.betaCGD
    xd = OPS.pool2(x)
    t = OPS.system_half(xd, wL1, cG1, m.GLRmodule01, m.GTVmodule01, m.muys01, m.ro01, g)
    ref1, u1, xd1 = OPS.system_step(x, b, u, t, wL0, cG0, m.GLRmodule00, m.GTVmodule00, m.muys00, m.ro00, alpha[k],
                                    beta[k] if u is not None else None, g, want_u=True, want_pool=True)
    t1 = OPS.system_half(xd1, wL1, cG1, m.GLRmodule01, m.GTVmodule01, m.muys01, m.ro01, g)
    ref2, u2, xd2 = OPS.system_step(ref1, b, u1, t1, wL0, cG0, m.GLRmodule00, m.GTVmodule00, m.muys00, m.ro00,
                                    alpha[k + 1], beta[k + 1], g, want_u=not last, want_pool=not last,
                                    skip=skip, y_skip=y_skip)
    got, gu, gxd = OPS.system_step2(x, b, u, xd, wL0, cG0, m.GLRmodule00, m.GTVmodule00, m.muys00, m.ro00, wL1, cG1,
                                    m.GLRmodule01, m.GTVmodule01, m.muys01, m.ro01, alpha[k],
                                    beta[k] if u is not None else None, alpha[k + 1], beta[k + 1], g,
                                    want_u=not last, want_pool=not last, skip=skip, y_skip=y_skip)
    return (ref2, u2, xd2), (got, gu, gxd)


CASES = [
    dict(B=2, G=4, F=3, H=256),     # segmented grid: 64-row segments
    dict(B=16, G=32, F=3, H=256),   # one segment per (b, graph): the bench's workgroup shape
    dict(B=3, G=2, F=3, H=16),      # shorter than the pipeline lag
    dict(B=2, G=3, F=2, H=130),     # H not a multiple of the segment, F = 2
    dict(B=1, G=4, F=1, H=64),
    dict(B=2, G=2, F=3, H=8),       # half rows fewer than the half-level pipeline's fill
    dict(B=2, G=2, F=6, H=64),      # v1.0 first filter block: two channel groups of 3
    dict(B=1, G=2, F=12, H=32),     # four groups of 3
    dict(B=1, G=3, F=5, H=32),      # uneven groups (3 + 2)
]


STRIP_CASES = [
    dict(B=2, G=4, F=3, H=64, W=496),    # three strips (the 336 x 496 evaluation pad, landscape)
    dict(B=1, G=3, F=3, H=96, W=336),    # two strips (portrait)
    dict(B=2, G=2, F=6, H=32, W=512),    # C4's width, channel groups
    dict(B=1, G=2, F=2, H=16, W=744),    # four strips
    dict(B=2, G=4, F=3, H=256, W=480),   # two strips, last strip 32 columns short of its window
    dict(B=2, G=2, F=3, H=32, W=128),    # one strip, half the lanes past the edge
    dict(B=1, G=2, F=3, H=12, W=200),
    dict(B=1, G=2, F=1, H=8, W=8),       # one lane of image
]


@pytest.mark.parametrize("case", CASES + STRIP_CASES, ids=lambda c: "b{B}g{G}f{F}h{H}w{W}".format(W=256, **c)
                         if "W" not in c else "b{B}g{G}f{F}h{H}w{W}".format(**c))
@pytest.mark.parametrize("with_u", [True, False])
def test_step2_equals_two_steps(irdu, case, with_u):
    B, G, F, H = case["B"], case["G"], case["F"], case["H"]
    mix, x, b, u, w = _setup(irdu, B, G, F, H, seed=B * 100 + H + F, W=case.get("W", 256))
    with torch.no_grad():
        (r, ru, rxd), (o, ou, oxd) = _two_steps(irdu, mix, x, b, u if with_u else None, w, k=2, g=G)
    torch.cuda.synchronize()
    for name, a, bb in (("x", o, r), ("u", ou, ru), ("xd", oxd, rxd)):
        e = rel_err(a, bb)
        assert e <= TIGHT, (name, e)
        assert torch.isfinite(a).all()


def test_step2_last_pair_with_skip(irdu):
    mix, x, b, u, w = _setup(irdu, 2, 4, 3, 256, seed=77)
    y = torch.rand_like(x)
    skip = torch.tensor([0.7, 0.4], device=DEV)
    with torch.no_grad():
        (r, ru, rxd), (o, ou, oxd) = _two_steps(irdu, mix, x, b, u, w, k=2, g=4, skip=skip, y_skip=y, last=True)
    assert ou is None and oxd is None and ru is None and rxd is None
    assert rel_err(o, r) <= TIGHT


def test_step2_rejects_unsupported_shapes(irdu):
    from irdu_amd import kernels as K
    from irdu_amd._native import GrrError
    mix, x, b, u, w = _setup(irdu, 1, 2, 3, 16, seed=5)
    xs = x[..., :132].contiguous()   # W % 8 != 0
    wL0, cG0, wL1, cG1 = w
    m = mix
    with pytest.raises(GrrError):
        K.system_step2(xs, xs, None, torch.zeros(1, 6, 8, 66, device=DEV), wL0[..., :132].contiguous(),
                       cG0[..., :132].contiguous(), K.stencil(m.GLRmodule00), K.stencil(m.GTVmodule00), m.muys00,
                       m.ro00, wL1[..., :66].contiguous(), cG1[..., :66].contiguous(), K.stencil(m.GLRmodule01),
                       K.stencil(m.GTVmodule01), m.muys01, m.ro01, m.alphaCGD[0], None, m.alphaCGD[1],
                       m.betaCGD[1], 2, True, True)
    assert not K.step2_supported(xs, 2)
    assert K.step2_supported(x[..., :128], 2) == (K.STEP2_STRIPS and K.STEP2_MIN_W <= 128)
    assert not K.step2_supported(x[..., :64], 2) or K.STEP2_MIN_W <= 64   # W = 64: per-stage kernels
    assert K.step2_supported(torch.empty(1, 6, 16, 496, device="meta"), 2) == K.STEP2_STRIPS


@pytest.mark.parametrize("b,hw", [(1, (256, 256)), (3, (256, 256)), (1, (336, 496)), (1, (496, 336))])
def test_filter_with_step2_matches_per_stage_launches_and_oracle(irdu, b, hw):
    """The image filter (S = 10: stage 0, then pairs (1,2) ... (7,8) and stage 9) with and without
    two-stage launches, and against the CPU oracle at the PSNR tolerance; 336 x 496 / 496 x 336 is the
    reference's CBSD68 evaluation pad (column strips)."""
    from irdu_amd import kernels as K
    torch.manual_seed(2300 + b)
    m = irdu.MultiScaleGraphFilter(3, 3, ngraphs=8, n_cgd_iters=10)
    perturb_mixture(m.localfilter, 23 + b)
    clean = torch.rand(b, 3, *hw)
    noisy = clean + torch.randn(b, 3, *hw) * (25.0 / 255.0)
    md = m.to(DEV)
    saved = K.STEP2
    try:
        with torch.no_grad():
            K.STEP2 = True
            fused = md(noisy.to(DEV)).cpu()
            K.STEP2 = False
            single = md(noisy.to(DEV)).cpu()
    finally:
        K.STEP2 = saved
    assert rel_err(fused, single) <= 1e-5
    ref = O.multiscale_graph_filter(noisy, sd_cpu(m), 8)
    assert rel_err(fused, ref) <= 1e-4
    assert abs(O.psnr_ubyte(fused, clean) - O.psnr_ubyte(ref, clean)) <= 0.01


@pytest.mark.parametrize("n_st,w", [(4, 256), (5, 256), (5, 512)])
def test_training_forward_with_step2_matches_per_stage(irdu, n_st, w):
    """The training forward (grr_system_step2_train: pairs that also write the middle iterate for the
    reverse sweep) against one stage per launch: output, loss gradient of the input and of every
    parameter of the image filter (S = 4: pair (1,2) + stage 3; S = 5: pairs (1,2), (3,4))."""
    from irdu_amd import kernels as K
    torch.manual_seed(2400 + n_st)
    m = irdu.MultiScaleGraphFilter(3, 3, ngraphs=4, n_cgd_iters=n_st)
    perturb_mixture(m.localfilter, 24 + n_st)
    x = torch.rand(2, 3, 32, w)
    gout = torch.randn(2, 3, 32, w)
    md = m.to(DEV).train()
    saved = K.STEP2
    res = {}
    try:
        for flag in (True, False):
            K.STEP2 = flag
            md.zero_grad(set_to_none=True)
            xd = x.to(DEV).requires_grad_(True)
            out = md(xd)
            out.backward(gout.to(DEV))
            res[flag] = (out.detach().cpu(), xd.grad.cpu(),
                         {k: p.grad.detach().cpu() for k, p in md.named_parameters() if p.grad is not None})
    finally:
        K.STEP2 = saved
    (o1, g1, p1), (o0, g0, p0) = res[True], res[False]
    assert rel_err(o1, o0) <= 1e-5
    assert rel_err(g1, g0) <= 1e-5
    assert p1.keys() == p0.keys()
    for k in p0:
        assert rel_err(p1[k], p0[k]) <= 1e-4, k


def test_training_step2_mid_pool_equals_pool2(irdu):
    """grr_system_step2_train's xd_mid (D x_{k+1}, the pooled rows stage B's half level reads) against
    grr_pool2 of the middle iterate it writes; without xd_mid the other outputs are unchanged."""
    from irdu_amd import kernels as K
    torch.manual_seed(77)
    G, F, B, H, W = 4, 3, 2, 64, 256
    m = irdu.MixtureGTVGLR(G, F, 0.5, 0.1, [[1e-3], [1e-4]], [[1e-4], [1e-4]], [[1e-4], [1e-4]], n_cgd_iters=10)
    perturb_mixture(m, 77)
    m = m.to(DEV)
    f0 = torch.randn(B, 2 * G * F, H, W, device=DEV)
    f1 = torch.randn(B, 2 * G * F, H // 2, W // 2, device=DEV)
    wG0, cG0, wL0 = K.edge_weights_block(f0, G, F, m.GTVmodule00.multiM, m.GLRmodule00.multiM)
    wG1, cG1, wL1 = K.edge_weights_block(f1, G, F, m.GTVmodule01.multiM, m.GLRmodule01.multiM)
    x = torch.rand(B, G * F, H, W, device=DEV)
    rhs = torch.rand_like(x)
    u = torch.randn_like(x)
    xd = K.pool2(x)
    args = (x, rhs, u, xd, wL0, cG0, K.stencil(m.GLRmodule00), K.stencil(m.GTVmodule00), m.muys00, m.ro00, wL1,
            cG1, K.stencil(m.GLRmodule01), K.stencil(m.GTVmodule01), m.muys01, m.ro01, m.alphaCGD[2],
            m.betaCGD[2], m.alphaCGD[3], m.betaCGD[3], G)
    with torch.no_grad():
        got = K.system_step2_train(*args, want_pool=True, want_mid_pool=True)
        ref = K.system_step2_train(*args, want_pool=True, want_mid_pool=False)
    torch.cuda.synchronize()
    assert ref[5] is None
    for a, r in zip(got[:5], ref[:5]):
        assert torch.equal(a, r)
    assert rel_err(got[5], K.pool2(got[0])) <= 1e-6


@pytest.mark.parametrize("n_st", [4, 5])
def test_training_saved_pooled_iterates_match_repooling(irdu, n_st):
    """solver_grad.SAVE_POOLED (the reverse's half level reads D x_k saved by the forward) against
    pooling the saved iterates in the reverse: input and parameter gradients."""
    from irdu_amd import solver_grad as SG
    torch.manual_seed(2500 + n_st)
    m = irdu.MultiScaleGraphFilter(3, 3, ngraphs=4, n_cgd_iters=n_st)
    perturb_mixture(m.localfilter, 25 + n_st)
    x = torch.rand(2, 3, 32, 256)
    gout = torch.randn(2, 3, 32, 256)
    md = m.to(DEV).train()
    saved = SG.SAVE_POOLED
    res = {}
    try:
        for flag in (True, False):
            SG.SAVE_POOLED = flag
            md.zero_grad(set_to_none=True)
            xd = x.to(DEV).requires_grad_(True)
            out = md(xd)
            out.backward(gout.to(DEV))
            res[flag] = (out.detach().cpu(), xd.grad.cpu(),
                         {k: p.grad.detach().cpu() for k, p in md.named_parameters() if p.grad is not None})
    finally:
        SG.SAVE_POOLED = saved
    (o1, g1, p1), (o0, g0, p0) = res[True], res[False]
    assert torch.equal(o1, o0)
    assert rel_err(g1, g0) <= 1e-5
    for k in p0:
        assert rel_err(p1[k], p0[k]) <= 1e-4, k
