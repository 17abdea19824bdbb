"""``model.compile()`` maps the default Inductor backend to ``irdu_hip`` (compile_backend.py): AOTAutograd
graphs run node by node, nothing is code-generated.  On CPU Inductor would generate C++ kernels for the
stock ops of the v1.0 encoder / decoder (3x3 replicate conv, 2x2 down / up convs, cat, 1x1 combine), so
a zero ``generated_kernel_count`` after a compiled forward + backward shows Inductor never ran.  The
graph-filter ops themselves are opaque irdu:: nodes (tests/test_compile_training.py); the compiled GPU
training step is tests/test_gpu_compile.py."""
import torch
import torch.nn.functional as F

import irdu_amd
from irdu_amd import compile_backend as CB
from irdu_amd.graph_filter import Downsampling, ReginalPixelEmbeding, Upsampling


class _EncDec(CB.HipModule):
    """The v1.0 model's stock (non-HIP) layers: embedding, 2x2/s2 down, 2x2 transposed up, cat + 1x1."""

    def __init__(self):
        super().__init__()
        self.emb = ReginalPixelEmbeding(3, 8)
        self.down = Downsampling(8, 16, 1)
        self.up = Upsampling(16, 8, 1)
        self.comb = torch.nn.Conv2d(16, 8, 1, bias=False)
        self.out = torch.nn.Conv2d(8, 3, 1, bias=False)

    def forward(self, x):
        e = self.emb(x)
        return self.out(self.comb(torch.cat([self.up(self.down(e)), e], 1)))


def _step(m, x, c):
    loss = F.l1_loss(m(x), c) + 0.1 * F.mse_loss(m(c), c)
    loss.backward()
    return float(loss.detach()), {k: p.grad.clone() for k, p in m.named_parameters()}


def test_default_backend_is_mapped():
    assert CB.resolve({})["backend"] == CB.BACKEND
    assert CB.resolve({"backend": "inductor", "mode": "max-autotune"}) == {"backend": CB.BACKEND}
    assert CB.resolve({"backend": "cudagraphs"})["backend"] == "cudagraphs"
    for cls in (irdu_amd.AbtractMultiScaleGraphFilter, irdu_amd.MultiScaleGraphFilter, irdu_amd.MixtureGTVGLR,
                irdu_amd.LocalNonLinearBlock, irdu_amd.GLRFast, irdu_amd.GTVFast, irdu_amd.MultiScaleGLRImageFilter,
                irdu_amd.window_graph.MultiScaleSequenceDenoiser, irdu_amd.window_graph_v1.MultiScaleSequenceDenoiser):
        assert issubclass(cls, CB.HipModule), cls


def test_module_compile_generates_no_kernels_and_matches_eager():
    import torch._inductor.metrics as metrics
    torch._dynamo.reset()
    torch.manual_seed(0)
    x, c = torch.rand(2, 3, 16, 16), torch.rand(2, 3, 16, 16)
    ref = _EncDec()
    m = _EncDec()
    m.load_state_dict(ref.state_dict())
    ref_loss, ref_grads = _step(ref, x, c)
    metrics.reset()
    m.compile()
    loss, grads = _step(m, x, c)
    assert metrics.generated_kernel_count == 0
    assert abs(loss - ref_loss) <= 1e-6 * abs(ref_loss)
    for k, g in ref_grads.items():
        assert torch.allclose(grads[k], g, rtol=1e-5, atol=1e-7), k


def test_inductor_would_generate_here():
    """Control: the same module under plain torch.compile (Inductor) does generate code on this
    host, so the zero above is a property of the mapping, not of the model."""
    import torch._inductor.metrics as metrics
    torch._dynamo.reset()
    torch.manual_seed(0)
    m = _EncDec()
    metrics.reset()
    torch.compile(m)(torch.rand(2, 3, 16, 16)).sum().backward()
    assert metrics.generated_kernel_count > 0
