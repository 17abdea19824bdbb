"""``model.compile()`` on the drop-in models (the reference compiles its model,
scripts_v2/run_abtract_lightformer_GGTV_GGLR_sigma25.py:130): the compiled forward runs the same
HIP kernels as eager -- every launch is an opaque irdu:: custom op (irdu_amd/ops.py) -- so the
outputs are bit-identical, and Inductor generates no kernels of its own for the graph-filter
models (no Triton).  The HIP-graph backend ("cudagraphs": capture + replay of the launch
sequence, no code generation) gives the same result.
"""
import pytest
import torch

from tests.test_gpu_parity import DEV, perturb_mixture

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def irdu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import irdu_amd
    irdu_amd.load_native()
    return irdu_amd


def _models(irdu):
    torch.manual_seed(11)
    msgf = irdu.MultiScaleGraphFilter(3, 3, ngraphs=8, n_cgd_iters=10)
    perturb_mixture(msgf.localfilter, 12)
    blk = irdu.LocalLowpassFilteringBlock(dim=48, nsubnets=1, ngraphs=8, n_cgd_iters=10)
    perturb_mixture(blk.local_filter, 13)
    return [("msgf", msgf, (2, 3, 64, 96)), ("lowpass", blk, (2, 48, 32, 64)),
            ("glr2", irdu.MultiScaleGLRImageFilter(1, 1, ngraphs=8, n_cgd_iters=5), (4, 1, 64, 64))]


@pytest.mark.parametrize("idx", [0, 1, 2])
def test_model_compile_matches_eager_without_codegen(irdu, idx):
    import torch._inductor.metrics as metrics
    torch._dynamo.reset()
    name, m, shape = _models(irdu)[idx]
    m = m.to(DEV).eval()
    x = torch.rand(*shape, device=DEV)
    with torch.no_grad():
        ref = m(x)
        metrics.reset()
        m.compile()                      # nn.Module.compile: default backend (Inductor)
        got = m(x)
        got2 = m(x)
    assert torch.equal(got, ref), name
    assert torch.equal(got2, ref), name
    assert metrics.generated_kernel_count == 0, f"{name}: Inductor generated {metrics.generated_kernel_count} kernels"


def test_hip_graph_backend_matches_eager(irdu):
    torch._dynamo.reset()
    _, m, shape = _models(irdu)[0]
    m = m.to(DEV).eval()
    x = torch.rand(*shape, device=DEV)
    with torch.no_grad():
        ref = m(x)
        cm = torch.compile(m, backend="cudagraphs")
        outs = [cm(x).clone() for _ in range(3)]   # warm-up, record, replay
    for o in outs:
        assert torch.equal(o, ref)
