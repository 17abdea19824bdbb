"""The reverse's reduction scratch under HIP-graph capture (graph_bwd.hip scratch_lease).

A reduction captured into a graph takes its own scratch (hipMallocAsync / hipFreeAsync memory nodes
of the graph), not the capturing stream's grow-only buffer: a replay running next to eager calls on
the same stream must not share their partial sums, and grr_release_scratch must not free memory the
graph still uses."""
import pytest
import torch

pytestmark = pytest.mark.gpu

B, G, F, H, W = 2, 3, 2, 24, 40


def _ref(u, v):
    return (u.double() * v.double()).view(B, G, F, H, W).sum((0, 2, 3, 4))


def test_captured_reduction_replays_beside_eager_calls():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import irdu_amd
    from irdu_amd import _native
    from irdu_amd import kernels as K
    irdu_amd.load_native()
    dev = torch.device("cuda:0")
    gen = torch.Generator().manual_seed(11)

    def rnd():
        return torch.randn(B, G * F, H, W, generator=gen).to(dev)

    u, v = rnd(), rnd()
    out = torch.zeros(G, device=dev)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):   # warm-up outside the capture (the stream's own buffer exists now)
        K.bwd_graph_dot(u, v, out, G)
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out.zero_()
        K.bwd_graph_dot(u, v, out, G)
    for it in range(4):
        u.copy_(rnd())
        v.copy_(rnd())
        graph.replay()
        # eager reductions on the replay's stream, queued right behind it, with other operands
        u2, v2 = rnd(), rnd()
        o2 = torch.zeros(G, device=dev)
        K.bwd_graph_dot(u2, v2, o2, G)
        K.bwd_graph_dot(u2, v2, o2, G, coef=-0.5)
        torch.cuda.synchronize()
        want = _ref(u, v)
        assert torch.allclose(out.double().cpu(), want.cpu(), rtol=1e-5, atol=1e-3), (it, out, want)
        assert torch.allclose(o2.double().cpu(), 0.5 * _ref(u2, v2).cpu(), rtol=1e-5, atol=1e-3), it
        if it == 1:
            _native.release_scratch()   # frees the streams' buffers, never the graph's own scratch
    del graph
    torch.cuda.synchronize()
