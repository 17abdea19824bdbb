"""The image filter's half-resolution feature branch (2x2 conv, LocalNonLinearBlocks, 1x1, the
half level's edge weights and its rhs-A term) runs on a second HIP stream beside the
full-resolution branch (graph_filter.FEATURE_STREAMS).  The kernels are deterministic, so the
two-stream forward must equal the one-stream forward bit for bit, for the replicated-RGB
MultiScaleGraphFilter and for a MixtureGTVGLR called on a plain signal."""
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


def _both(run):
    from irdu_amd import graph_filter as GF
    saved = GF.FEATURE_STREAMS
    try:
        outs = []
        for on in (False, True):
            GF.FEATURE_STREAMS = on
            with torch.no_grad():
                outs.append(run())
            torch.cuda.synchronize()
        return outs
    finally:
        GF.FEATURE_STREAMS = saved


def test_msgf_two_streams_bitwise(irdu):
    torch.manual_seed(7)
    m = irdu.MultiScaleGraphFilter(3, 3, ngraphs=8, n_cgd_iters=4).to(DEV)
    x = torch.rand(3, 3, 64, 96, device=DEV)
    a, b = _both(lambda: m(x))
    assert torch.equal(a, b)


def test_mixture_two_streams_bitwise(irdu):
    torch.manual_seed(8)
    g, f = 4, 3
    mix = irdu.MixtureGTVGLR(g, f, 0.5, 0.1, [[1e-1], [1e-2]], [[1e-1], [1e-2]], [[1e-2], [1e-2]],
                             n_cgd_iters=5, feature_extractor="v13").to(DEV)
    y = torch.rand(2, g * f, 48, 64, device=DEV)
    a, b = _both(lambda: mix(y))
    assert torch.equal(a, b)


def _assert_steps_close(g1, g2, w1, w2, bitwise=False):
    """Per parameter: 1e-5 relative to its own largest gradient + 1e-12 (the round-2 floor: the
    reductions are fixed-order now, so no summation-order noise); bitwise for the all-HIP msgf model
    (the stock convolutions' library reverses of the v1.0 model may reduce in any order)."""
    for step_a, step_b in zip(g1, g2):
        for a, b in zip(step_a, step_b):
            if a is None:
                assert b is None
                continue
            if bitwise:
                assert torch.equal(a, b)
            assert float((a - b).abs().max()) <= 1e-5 * float(b.abs().max()) + 1e-12
    for a, b in zip(w1, w2):
        if bitwise:
            assert torch.equal(a, b)
        assert float((a - b).abs().max()) <= 1e-5 * float(b.abs().max()) + 1e-12


def test_msgf_training_side_stream_matches_one_stream(irdu):
    """GRR_FEATURE_STREAMS_TRAIN: the half-resolution branch's forward and (autograd's stream replay)
    reverse on the side stream.  Three training steps (loss, backward, parameter update) per mode so
    the caching allocator recycles the cross-stream blocks; gradients and weights equal the one-stream
    run bit for bit (the kernels are deterministic and their reductions fixed-order)."""
    import torch.nn.functional as F
    from irdu_amd import graph_filter as GF

    def run(on):
        GF.FEATURE_STREAMS_TRAIN = on
        torch.manual_seed(9)
        m = irdu.MultiScaleGraphFilter(3, 3, ngraphs=8, n_cgd_iters=4).to(DEV).train()
        opt = torch.optim.SGD(m.parameters(), lr=1e-3)
        g = torch.Generator().manual_seed(3)
        grads = []
        for _ in range(3):
            x = torch.rand(2, 3, 64, 64, generator=g).to(DEV)
            t = torch.rand(2, 3, 64, 64, generator=g).to(DEV)
            opt.zero_grad(set_to_none=True)
            F.l1_loss(m(x), t).backward()
            grads.append([p.grad.clone() for p in m.parameters()])
            opt.step()
        torch.cuda.synchronize()
        return grads, [p.detach().clone() for p in m.parameters()]

    saved = GF.FEATURE_STREAMS_TRAIN
    try:
        (g1, w1), (g2, w2) = run(False), run(True)
    finally:
        GF.FEATURE_STREAMS_TRAIN = saved
    _assert_steps_close(g1, g2, w1, w2, bitwise=True)


@pytest.mark.parametrize("model", ["msgf", "abstract"])
def test_training_level_streams_match_one_stream(irdu, model):
    """solver_grad.LEVEL_STREAMS: the half level's reverse of every stage on a second stream beside the
    full level's.  Three training steps per mode (allocator recycling across streams); gradients and
    weights equal the one-stream run's: bitwise for msgf, to 1e-5 relative for the v1.0 model (its stock
    convolutions' library reverses)."""
    import torch.nn.functional as F
    from irdu_amd import solver_grad as SG

    def build():
        if model == "msgf":
            return irdu.MultiScaleGraphFilter(3, 3, ngraphs=8, n_cgd_iters=4)
        return irdu.AbtractMultiScaleGraphFilter(
            3, 3, dims=[8, 16, 16, 32], hidden_dims=[16, 32, 32, 64], nsubnets=[1, 1, 1, 1], ngraphs=[2, 4, 4, 8],
            num_blocks=[1, 1, 1, 1], num_blocks_out=1, n_cgd_iters=3)

    def run(on):
        SG.LEVEL_STREAMS = on
        torch.manual_seed(11)
        m = build().to(DEV).train()
        opt = torch.optim.SGD(m.parameters(), lr=1e-3)
        g = torch.Generator().manual_seed(5)
        grads = []
        for _ in range(3):
            x = torch.rand(2, 3, 64, 64, generator=g).to(DEV)
            t = torch.rand(2, 3, 64, 64, generator=g).to(DEV)
            opt.zero_grad(set_to_none=True)
            F.l1_loss(m(x), t).backward()
            grads.append([p.grad.clone() if p.grad is not None else None for p in m.parameters()])
            opt.step()
        torch.cuda.synchronize()
        return grads, [p.detach().clone() for p in m.parameters()]

    saved = SG.LEVEL_STREAMS
    try:
        (g1, w1), (g2, w2) = run(False), run(True)
    finally:
        SG.LEVEL_STREAMS = saved
    _assert_steps_close(g1, g2, w1, w2, bitwise=model == "msgf")


@pytest.mark.parametrize("model", ["msgf", "abstract"])
def test_lnb_kept_gate_matches_recompute(irdu, model):
    """solver_grad.KEEP_GATE: the eager LocalNonLinearBlock forward keeps the head's gated activation for
    the reverse's W2 weight gradient instead of recomputing depthwise + gate from W1 LN(x).  The kept
    gate comes from the fused head (fp16 two-term GEMM1), the recomputed one from the split-bf16 1x1
    GEMM: equal to fp32 accuracy, so the gradients agree to 1e-5 relative."""
    import torch.nn.functional as F
    from irdu_amd import solver_grad as SG

    def build():
        if model == "msgf":
            return irdu.MultiScaleGraphFilter(3, 3, ngraphs=8, n_cgd_iters=4)
        return irdu.AbtractMultiScaleGraphFilter(
            3, 3, dims=[8, 16, 16, 32], hidden_dims=[16, 32, 32, 64], nsubnets=[1, 1, 1, 1], ngraphs=[2, 4, 4, 8],
            num_blocks=[1, 1, 1, 1], num_blocks_out=1, n_cgd_iters=3)

    def run(keep):
        SG.KEEP_GATE = keep
        torch.manual_seed(13)
        m = build().to(DEV).train()
        g = torch.Generator().manual_seed(6)
        x = torch.rand(2, 3, 64, 64, generator=g).to(DEV)
        t = torch.rand(2, 3, 64, 64, generator=g).to(DEV)
        F.l1_loss(m(x), t).backward()
        torch.cuda.synchronize()
        return [p.grad.clone() if p.grad is not None else None for p in m.parameters()], SG._KEPT[0]

    saved = SG.KEEP_GATE
    try:
        (g0, _), (g1, kept_after) = run(False), run(True)
    finally:
        SG.KEEP_GATE = saved
    assert kept_after == 0          # every kept gate left the budget with its saved tensor
    for a, b in zip(g1, g0):
        if b is None:
            assert a is None
            continue
        assert float((a - b).abs().max()) <= 1e-5 * float(b.abs().max()) + 1e-12
