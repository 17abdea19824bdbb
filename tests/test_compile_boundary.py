"""The torch.library boundary (irdu_amd/ops.py) on CPU: every HIP entry point the inference
forwards launch is a registered custom op with a fake (meta) kernel, so a strict whole-graph
capture (torch.export, what torch.compile's Dynamo front end sees) of each drop-in model
contains only ``irdu::*`` ops and views -- nothing Inductor would generate code for, and no
graph break into the ctypes launch.  Nothing runs a kernel here (fake tensors only); the GPU
counterpart (tests/test_gpu_compile.py) runs ``model.compile()`` for real.
"""
import pytest
import torch

import irdu_amd
from irdu_amd import ops as OPS

# ops allowed besides irdu::*: views / indexing, no compute
VIEW_OPS = {"aten.view.default", "aten.select.int", "aten.reshape.default", "aten.unsqueeze.default",
            "aten.slice.Tensor", "<built-in function getitem>", "aten.detach.default", "aten.alias.default"}


def graph_ops(model, *args):
    with torch.no_grad():
        ep = torch.export.export(model.eval(), args, strict=True)
    seen = {}
    for n in ep.graph.nodes:
        if n.op == "call_function":
            seen[str(n.target)] = seen.get(str(n.target), 0) + 1
    return seen


def assert_only_irdu(seen):
    other = {k: v for k, v in seen.items() if not k.startswith("irdu.") and k not in VIEW_OPS}
    assert not other, f"non-irdu compute in the captured graph: {other}"
    assert any(k.startswith("irdu.") for k in seen)


def test_custom_ops_registered():
    for op in OPS.OPS:
        name = op._qualname.split("::")[1]
        assert hasattr(torch.ops.irdu, name), name


def test_msgf_graph_is_opaque_hip_ops():
    torch.manual_seed(0)
    m = irdu_amd.MultiScaleGraphFilter(3, 3, ngraphs=4, n_cgd_iters=4)
    seen = graph_ops(m, torch.rand(2, 3, 16, 24))
    assert_only_irdu(seen)
    assert seen["irdu.system_step.default"] == 4 and seen["irdu.system_half.default"] == 4
    assert seen["irdu.lnb_forward_rep.default"] == 1 and seen["irdu.lnb_forward.default"] == 5


@pytest.mark.parametrize("model_fn, shape", [
    (lambda: irdu_amd.LocalLowpassFilteringBlock(dim=12, nsubnets=1, ngraphs=4, n_cgd_iters=3), (1, 12, 16, 16)),
    (lambda: irdu_amd.MultiScaleGLRImageFilter(1, 1, ngraphs=8, n_cgd_iters=5), (2, 1, 32, 32)),
    (lambda: irdu_amd.GLRImageFilter(1, 1, ngraphs=4, n_cgd_iters=1), (1, 1, 64, 64)),
    (lambda: irdu_amd.v10.LocalLowpassFilteringBlock(dim=12, nsubnets=1, ngraphs=4), (1, 12, 16, 16)),
    (lambda: irdu_amd.LocalNonLinearBlock(16, 32, 1), (1, 16, 8, 8)),
])
def test_model_graphs_are_opaque_hip_ops(model_fn, shape):
    torch.manual_seed(1)
    assert_only_irdu(graph_ops(model_fn(), torch.rand(*shape)))


class _SubApi(torch.nn.Module):
    """Composes the GLRFast / GTVFast module methods the way REF:218-237 / :518-523 do."""

    def __init__(self, f, g):
        super().__init__()
        self.glr = irdu_amd.GLRFast(f, g, 1.0)
        self.gtv = irdu_amd.GTVFast(f, g, 1.0)

    def forward(self, feat, x):
        w, d = self.glr.extract_edge_weights(feat)
        b, g, f, h, ww = x.shape
        nb = self.glr.get_neighbors_pixels(x.reshape(b, g * f, h, ww))
        n = self.glr.normalize_and_transform_features(feat)
        l = self.glr.stats_conv_transpose(self.glr.op_L_norm(self.glr.stats_conv(x), w, d))
        e = self.gtv.op_C(x, w, d)
        return l, self.gtv.op_C_transpose(e, w, d), self.gtv(x, w, d), self.glr(x, w, d), nb, n


def test_sub_api_graph_is_opaque_hip_ops():
    f, g = 3, 2
    seen = graph_ops(_SubApi(f, g), torch.rand(1, g, f, 8, 10), torch.rand(1, g, f, 8, 10))
    assert_only_irdu(seen)
    for name in ("neighbor_gather", "normalize_features", "stats_conv", "glr_op_L_norm", "gtv_op_C",
                 "gtv_op_C_transpose", "edge_weights", "gtv_pair_weights", "system_half"):
        assert f"irdu.{name}.default" in seen, name


def test_eager_path_bypasses_dispatcher():
    """Outside tracing the helpers call kernels directly (no dispatcher hop per launch); on CPU the
    kernels refuse the tensor, which is the engine's loud no-fallback behaviour."""
    with pytest.raises(RuntimeError, match="no CPU path"):
        OPS.pool2(torch.rand(1, 1, 4, 4))
