"""grr_system_first_pair (stage 0, the prox right-hand side B and stage 1 in one pass; x_1 never leaves the
chip) against the launch sequence it replaces: grr_system_half -> grr_system_step (stage 0) ->
grr_gtv_rhs_half -> grr_gtv_rhs_full (prox: right-hand side B) -> grr_system_half -> grr_system_step
(stage 1), REF:751-790.  Same per-row arithmetic; 2e-6 relative to the largest output covers fp32
contraction differences between the two code paths.  Shapes: one row segment per (b, graph) and the
segmented grid (the stage-A lead crossing segment boundaries), images shorter than the pipeline lag,
F > 3 as channel groups (uneven 3 + 2), y given in full or as the image it replicates over the graphs
(the image filter's src), soft thresholds with both branches active at both levels.  The image filter
(S = 10) with and without the pass is compared in test_gpu_step2.py's filter test (against the per-stage
path and the CPU oracle) and below."""
import math

import pytest
import torch

from tests.test_gpu_parity import DEV, perturb_mixture, rel_err

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
    mix = irdu.MixtureGTVGLR(G, F, 0.5, 0.1, [[1e-3], [1e-4]], [[1e-4], [1e-4]], [[1e-4], [1e-4]], n_cgd_iters=10)
    perturb_mixture(mix, seed)
    with torch.no_grad():   # scales large enough that both levels and both prox branches matter
        mix.muys00.fill_(-1.0)
        mix.ro00.fill_(-1.5)
        mix.muys01.fill_(-1.2)
        mix.ro01.fill_(-1.6)
        mix.gamma00.copy_(torch.log(torch.linspace(0.02, 0.2, G)))
        mix.gamma01.copy_(torch.log(torch.linspace(0.03, 0.15, G)))
    mix = mix.to(DEV)
    f0 = torch.randn(B, 2 * G * F, H, W, device=DEV)
    f1 = torch.randn(B, 2 * G * F, H // 2, W // 2, device=DEV)
    wG0, cG0, wL0 = K.edge_weights_block(f0, G, F, mix.GTVmodule00.multiM, mix.GLRmodule00.multiM)
    wG1, cG1, wL1 = K.edge_weights_block(f1, G, F, mix.GTVmodule01.multiM, mix.GLRmodule01.multiM)
    C = G * F
    b_a = torch.rand(B, C, H, W, device=DEV)
    return mix, b_a, (wG0, cG0, wL0, wG1, cG1, wL1)


def _both(irdu, mix, b_a, w, y, y_rep, g):
    from irdu_amd import ops as OPS
    m = mix
    wG0, cG0, wL0, wG1, cG1, wL1 = w
    alpha = m.alphaCGD
    xd_a = OPS.pool2(b_a)
    t0 = OPS.system_half(xd_a, wL1, cG1, m.GLRmodule01, m.GTVmodule01, m.muys01, m.ro01, g)
    x1, _, xd1 = OPS.system_step(b_a, b_a, None, t0, wL0, cG0, m.GLRmodule00, m.GTVmodule00, m.muys00, m.ro00,
                                 alpha[0], None, g, want_u=False, want_pool=True)
    tp = OPS.gtv_rhs_half(xd1, wG1, m.GTVmodule01, True, m.gamma01, g)
    b_b, _ = OPS.gtv_rhs_full(x1, False, y, y_rep, wG0, m.GTVmodule00, True, m.gamma00, m.ro00, tp, m.ro01, g)
    t1 = OPS.system_half(xd1, wL1, cG1, m.GLRmodule01, m.GTVmodule01, m.muys01, m.ro01, g)
    x2, u2, xd2 = OPS.system_step(x1, b_b, None, t1, wL0, cG0, m.GLRmodule00, m.GTVmodule00, m.muys00, m.ro00,
                                  alpha[1], None, g, want_u=True, want_pool=True)
    got = OPS.system_first_pair(b_a, xd_a, y, y_rep, wL0, cG0, wG0, m.GLRmodule00, m.GTVmodule00, m.muys00, m.ro00,
                                m.gamma00, wL1, cG1, wG1, m.GLRmodule01, m.GTVmodule01, m.muys01, m.ro01, m.gamma01,
                                alpha[0], alpha[1], g)
    return (b_b, x2, u2, xd2), got


CASES = [
    dict(B=2, G=4, F=3, H=256),     # segmented grid: 64-row segments
    dict(B=16, G=32, F=3, H=256),   # one segment per (b, graph): the bench's workgroup shape
    dict(B=3, G=2, F=3, H=16),      # shorter than the pipeline lag
    dict(B=2, G=3, F=2, H=130),     # H not a multiple of the segment, F = 2
    dict(B=1, G=4, F=1, H=64),
    dict(B=2, G=2, F=3, H=8),       # half rows fewer than the half-level pipeline's fill
    dict(B=2, G=2, F=6, H=64),      # v1.0 first filter block: two channel groups of 3
    dict(B=1, G=3, F=5, H=32),      # uneven groups (3 + 2)
    dict(B=1, G=2, F=3, H=2),       # one half row
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "b{B}g{G}f{F}h{H}".format(**c))
@pytest.mark.parametrize("y_rep", [False, True], ids=["y", "yrep"])
def test_first_pair_equals_launch_sequence(irdu, case, y_rep):
    B, G, F, H = case["B"], case["G"], case["F"], case["H"]
    mix, b_a, w = _setup(irdu, B, G, F, H, seed=B * 100 + H + F + (7 if y_rep else 0))
    if y_rep:
        y = torch.rand(B, F, H, 256, device=DEV)
    else:
        y = b_a + 0.1 * torch.randn_like(b_a)
    with torch.no_grad():
        ref, got = _both(irdu, mix, b_a, w, y, y_rep, G)
    torch.cuda.synchronize()
    for name, a, r in zip(("b_B", "x_2", "u_2", "D x_2"), got, ref):
        assert torch.isfinite(a).all(), name
        e = rel_err(a, r)
        assert e <= TIGHT, (name, e)


def test_first_pair_rejects_unsupported_shapes(irdu):
    from irdu_amd import kernels as K
    from irdu_amd._native import GrrError
    mix, b_a, w = _setup(irdu, 1, 2, 3, 16, seed=3)
    m = mix
    wG0, cG0, wL0, wG1, cG1, wL1 = w
    xs = b_a[..., :128].contiguous()
    with pytest.raises(GrrError):
        K.system_first_pair(xs, torch.zeros(1, 6, 8, 64, device=DEV), xs, False, wL0[..., :128].contiguous(),
                            cG0[..., :128].contiguous(), wG0[..., :128].contiguous(), K.stencil(m.GLRmodule00),
                            K.stencil(m.GTVmodule00), m.muys00, m.ro00, m.gamma00, wL1[..., :64].contiguous(),
                            cG1[..., :64].contiguous(), wG1[..., :64].contiguous(), K.stencil(m.GLRmodule01),
                            K.stencil(m.GTVmodule01), m.muys01, m.ro01, m.gamma01, m.alphaCGD[0], m.alphaCGD[1], 2)
    assert not K.first_pair_supported(xs, 2)
    assert K.first_pair_supported(b_a, 2) == K.FIRST_PAIR


@pytest.mark.parametrize("model", ["msgf", "lowpass"])
def test_filter_with_first_pair_matches_without(irdu, model):
    """The image filter (src replicated: y_rep) and a LocalLowpassFilteringBlock (full y, skip on the last
    pair) with the first-pair pass against stage 0 + rhs B + pairs (1,2) ... + stage S-1."""
    from irdu_amd import kernels as K
    torch.manual_seed(31 if model == "msgf" else 32)
    if model == "msgf":
        m = irdu.MultiScaleGraphFilter(3, 3, ngraphs=8, n_cgd_iters=10)
        perturb_mixture(m.localfilter, 41)
        x = torch.rand(2, 3, 64, 256)
    else:
        m = irdu.LocalLowpassFilteringBlock(dim=48, nsubnets=1, ngraphs=8, n_cgd_iters=10)
        perturb_mixture(m.local_filter, 42)
        x = torch.rand(2, 48, 32, 256)
    md = m.to(DEV).eval()
    saved = K.FIRST_PAIR
    try:
        with torch.no_grad():
            K.FIRST_PAIR = True
            fused = md(x.to(DEV)).cpu()
            K.FIRST_PAIR = False
            ref = md(x.to(DEV)).cpu()
    finally:
        K.FIRST_PAIR = saved
    assert math.isfinite(float(fused.abs().max()))
    assert rel_err(fused, ref) <= 1e-5


@pytest.mark.parametrize("bh", [(1, 256), (2, 130)], ids=["b1h256", "b2h130"])
def test_first_pair_f6_segmented_vs_oracle(irdu, bh):
    """MixtureGTVGLR at F = 6 (the v1.0 first filter block: two channel groups of 3), S = 10, W = 256 so the
    first-pair pass runs, on a segmented grid (B G groups far below the step-2 grid floor: 64-row segments at
    H = 256, a ragged last segment at H = 130) against the CPU oracle (REF:707-811) at the north_star
    tolerance (1e-4 normwise), not against the HIP launch sequence it replaces."""
    from oracle import graph_oracle as O
    from irdu_amd import kernels as K
    from tests.test_gpu_parity import assert_close, sd_cpu
    B, H = bh
    G, F = 2, 6
    torch.manual_seed(4600 + H)
    m = irdu.MixtureGTVGLR(G, F, 0.5, 0.1, [[1e-3], [1e-4]], [[1e-4], [1e-4]], [[1e-4], [1e-4]], n_cgd_iters=10)
    perturb_mixture(m, 46 + B)
    g = torch.Generator().manual_seed(46 + B)
    with torch.no_grad():   # mu, rho in [0.01, 0.06]: the ten-stage iteration stays bounded at F = 6 and
        for q in (m.muys00, m.muys01, m.ro00, m.ro01):   # still moves the output by ~0.2 (perturb_mixture's
            q.copy_(torch.log(0.01 + 0.05 * torch.rand(q.shape, generator=g)))   # 0.05-0.6 diverges here)
    x = torch.rand(B, G * F, H, 256)
    ref = O.mixture_forward(x, sd_cpu(m), G, "v1")
    md = m.to(DEV).eval()
    xd = x.to(DEV)
    assert K.first_pair_supported(xd, G) == K.FIRST_PAIR
    saved = K.FIRST_PAIR
    try:
        with torch.no_grad():
            K.FIRST_PAIR = True
            got = md(xd)
    finally:
        K.FIRST_PAIR = saved
    assert float(ref.abs().max()) < 2.0 and float((ref - x).abs().max()) > 0.05
    assert torch.isfinite(got).all()
    assert_close(got, ref)
