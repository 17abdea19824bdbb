"""The internal-stream invariant, checked (stream_guard.py): one msgf training step (feature branch on the
side stream, the solver reverse's half level on the level stream) and one inference forward run under
the guard without a violation, with ops actually observed on the internal streams; a library GEMM on
either stream -- in the forward or inside autograd's backward -- raises."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def irdu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import irdu_amd
    irdu_amd.load_native()
    return irdu_amd


def _msgf(irdu):
    from tests.test_gpu_parity import perturb_mixture
    torch.manual_seed(3)
    m = irdu.MultiScaleGraphFilter(3, 3, ngraphs=8, n_cgd_iters=4)
    perturb_mixture(m.localfilter, 5)
    return m.cuda()


def test_training_and_inference_steps_respect_the_invariant(irdu):
    from irdu_amd import graph_filter, solver_grad, training
    from irdu_amd.stream_guard import stream_guard
    assert graph_filter.FEATURE_STREAMS and graph_filter.FEATURE_STREAMS_TRAIN and solver_grad.LEVEL_STREAMS
    tr = training.Trainer(_msgf(irdu), {}, torch.device("cuda:0"))
    g = torch.Generator().manual_seed(1)
    clean = torch.rand(2, 64, 64, 3, generator=g)
    noisy = clean + 0.1 * torch.randn(2, 64, 64, 3, generator=g)
    with stream_guard() as mode:
        loss = tr.step(noisy, clean)
    torch.cuda.synchronize()
    assert loss == loss and mode.checked > 0
    with stream_guard() as mode, torch.no_grad():
        out = tr.model.eval()(noisy.permute(0, 3, 1, 2).contiguous().cuda())
    torch.cuda.synchronize()
    assert bool(torch.isfinite(out).all()) and mode.checked > 0


def test_library_gemm_on_an_internal_stream_raises(irdu):
    from irdu_amd import graph_filter, solver_grad
    from irdu_amd.stream_guard import StreamInvariantError, stream_guard
    dev = torch.device("cuda:0")
    a = torch.rand(64, 64, device=dev)
    for side in (graph_filter._side_stream(dev), solver_grad._level_side(dev)):
        side.wait_stream(torch.cuda.current_stream())
        with stream_guard():
            torch.mm(a, a)                                   # the caller's stream: allowed
            with torch.cuda.stream(side), pytest.raises(StreamInvariantError):
                torch.mm(a, a)
    torch.cuda.synchronize()


def test_violation_inside_backward_raises(irdu):
    from irdu_amd import graph_filter
    from irdu_amd.stream_guard import StreamInvariantError, stream_guard
    dev = torch.device("cuda:0")
    side = graph_filter._side_stream(dev)

    class Bad(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            return x * 2

        @staticmethod
        def backward(ctx, g):
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                h = g @ g.t()                                # a library GEMM on the side stream
            torch.cuda.current_stream().wait_stream(side)
            return h @ g

    x = torch.rand(32, 32, device=dev, requires_grad=True)
    with stream_guard(), pytest.raises(StreamInvariantError):
        Bad.apply(x).sum().backward()
    torch.cuda.synchronize()
