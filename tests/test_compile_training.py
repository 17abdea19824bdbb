"""``model.compile()`` + a training step (scripts_v2/run_abtract_lightformer_GGTV_GGLR_sigma25.py:130,
:186-207) on CPU, graphs only: the HIP forward and reverse of every differentiable graph-filter op
(solver_grad.py on train_ops.OpaqueFunction) reach AOTAutograd as opaque irdu:: nodes -- one in the
forward graph, its ``_backward`` twin in the backward graph -- so Inductor never sees (or generates
code for) them.  The recording backend returns zeros instead of running anything, so no kernel runs
here; tests/test_gpu_compile.py runs the compiled training step for real.
"""
import torch
import torch.nn.functional as F

import irdu_amd


def _record():
    from functorch.compile import make_boxed_func
    from torch._dynamo.backends.common import aot_autograd
    graphs = {"fw": [], "bw": []}

    def compiler(kind):
        def fn(gm, example_inputs):
            graphs[kind].append(gm)
            out_node = next(n for n in gm.graph.nodes if n.op == "output")
            vals = [a.meta.get("val") if isinstance(a, torch.fx.Node) else None for a in out_node.args[0]]

            def run(*args):
                return [None if v is None else torch.zeros(v.shape, dtype=v.dtype) for v in vals]
            return make_boxed_func(run)
        return fn

    return aot_autograd(fw_compiler=compiler("fw"), bw_compiler=compiler("bw")), graphs


def _targets(gms):
    seen = {}
    for gm in gms:
        for n in gm.graph.nodes:
            if n.op == "call_function":
                seen[str(n.target)] = seen.get(str(n.target), 0) + 1
    return seen


def _small_abstract(stages=3):
    torch.manual_seed(0)
    return irdu_amd.AbtractMultiScaleGraphFilter(
        3, 3, dims=[8, 16, 16, 32], hidden_dims=[16, 32, 32, 64], nsubnets=[1, 1, 1, 1], ngraphs=[2, 4, 4, 8],
        num_blocks=[1, 1, 1, 1], num_blocks_out=1, n_cgd_iters=stages)


def test_compiled_training_step_keeps_hip_ops_opaque():
    torch._dynamo.reset()
    backend, graphs = _record()
    m = _small_abstract().train()
    cm = torch.compile(m, backend=backend)
    x, c = torch.rand(2, 3, 32, 32), torch.rand(2, 3, 32, 32)
    loss = F.l1_loss(cm(x), c)
    loss.backward()
    fw, bw = _targets(graphs["fw"]), _targets(graphs["bw"])
    # four LocalLowpassFilteringBlocks, 1 + 1 + 1 + 1 encoder + 1 + 1 + 1 decoder + 1 refining LNBs
    assert fw.get("irdu.mixture_solve_train.default") == 4, fw
    assert bw.get("irdu.mixture_solve_train_backward.default") == 4, bw
    assert fw.get("irdu.lnb_train.default") == 8 and bw.get("irdu.lnb_train_backward.default") == 8
    assert fw.get("irdu.conv1x1_train.default") == 8 and fw.get("irdu.conv2x2s2_train.default") == 4
    # nothing of the solver was decomposed into aten ops the backend would compile
    for name in ("aten.softmax", "aten._softmax", "aten.linalg_vector_norm", "aten.where"):
        assert not any(k.startswith(name) for k in list(fw) + list(bw)), name
    for p in m.parameters():
        assert p.grad is not None


def test_compiled_msgf_and_glr_training_graphs():
    torch._dynamo.reset()
    backend, graphs = _record()
    torch.manual_seed(1)
    msgf = irdu_amd.MultiScaleGraphFilter(3, 3, ngraphs=4, n_cgd_iters=4).train()
    F.l1_loss(torch.compile(msgf, backend=backend)(torch.rand(1, 3, 16, 16)), torch.rand(1, 3, 16, 16)).backward()
    glr2 = irdu_amd.MultiScaleGLRImageFilter(1, 1, ngraphs=4, n_cgd_iters=3).train()
    F.l1_loss(torch.compile(glr2, backend=backend)(torch.rand(1, 1, 16, 16)), torch.rand(1, 1, 16, 16)).backward()
    fw, bw = _targets(graphs["fw"]), _targets(graphs["bw"])
    for op in ("mixture_solve_train", "lnb_train", "glr2_solve_train", "conv1x1_train", "conv2x2s2_train"):
        assert f"irdu.{op}.default" in fw, (op, fw)
        assert f"irdu.{op}_backward.default" in bw, (op, bw)
    # the input image needs no gradient: the replication's reverse is pruned from the backward graph
    assert "irdu.repeat_graphs_train.default" in fw and "irdu.repeat_graphs_train_backward.default" not in bw
