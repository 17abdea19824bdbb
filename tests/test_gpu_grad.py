"""GPU parity of the training path: gradients of the HIP reverse sweep (solver_grad.py,
graph_bwd.hip) against autograd through the CPU oracle run in float64.

Tolerance: max|grad_hip - grad_oracle| / max|grad_oracle| <= 2e-4 per tensor (fp32 HIP
vs fp64 oracle; the reductions over pixels / stages are fp32 with atomics).  The loss is
<out, R> with a fixed random R, so every output element carries gradient.
"""
import pytest
import torch

from oracle import graph_oracle as O
from tests.test_gpu_parity import DEV, perturb_mixture, rand, rel_err

pytestmark = pytest.mark.gpu

GTOL = 2e-4


@pytest.fixture(scope="module")
def irdu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import irdu_amd
    irdu_amd.load_native()
    return irdu_amd


def weights_r(shape):
    """The fixed random cotangent R (float32 draw, whatever the default dtype)."""
    g = torch.Generator().manual_seed(99)
    return torch.randn(*shape, generator=g, dtype=torch.float32)


def oracle_grads(fn, x, module):
    """Gradients of <fn(x, params), R> through the oracle in float64."""
    torch.set_default_dtype(torch.float64)
    try:
        params = {k: v.detach().cpu().double().requires_grad_(True) for k, v in module.state_dict().items()}
        xd = x.detach().cpu().double().requires_grad_(True)
        out = fn(xd, params)
        r = weights_r(out.shape).double()
        (out * r).sum().backward()
        return out.detach(), xd.grad, {k: v.grad for k, v in params.items()}
    finally:
        torch.set_default_dtype(torch.float32)


def hip_grads(module, x):
    module = module.to(DEV)
    module.zero_grad(set_to_none=True)
    xg = x.to(DEV).requires_grad_(True)
    out = module(xg)
    r = weights_r(out.shape).to(DEV)
    (out * r).sum().backward()
    torch.cuda.synchronize()
    return out.detach(), xg.grad, {k: p.grad for k, p in module.named_parameters()}


def check(module, fn, x, tol=GTOL, loose=()):
    """loose: parameter-name substrings held to 5e-2 instead of tol (see test_abstract_model_grad)."""
    ref_out, ref_gx, ref_gp = oracle_grads(fn, x, module)
    out, gx, gp = hip_grads(module, x)
    errs = {"out": rel_err(out, ref_out), "input": rel_err(gx, ref_gx)}
    for k, g in ref_gp.items():
        if g is None or float(g.abs().max()) == 0.0:
            continue
        assert gp.get(k) is not None, f"no gradient for {k}"
        errs[k] = rel_err(gp[k], g)
    worst = max(errs, key=errs.get)
    print(f"\n{type(module).__name__}: {len(errs)} tensors, worst rel err {errs[worst]:.2e} ({worst})")
    bad = {k: v for k, v in errs.items() if v > (5e-2 if any(s in k for s in loose) else tol)}
    assert not bad, f"gradients off: {bad}"
    return errs


@pytest.fixture(params=[True, False], ids=["fused", "multipass"])
def term_path(irdu, request):
    """Run a test with the one-pass fused term reverses and with the five-pass path."""
    from irdu_amd import solver_grad as SG
    SG.FUSED = request.param
    yield request.param
    SG.FUSED = True


@pytest.mark.parametrize("case", [dict(g=2, f=3, b=2, h=16, w=16, s=3), dict(g=4, f=2, b=1, h=12, w=20, s=5),
                                  dict(g=2, f=6, b=1, h=10, w=14, s=1), dict(g=3, f=3, b=1, h=18, w=8, s=10),
                                  dict(g=2, f=5, b=1, h=12, w=12, s=3),      # F = 5: no fused instance
                                  dict(g=2, f=12, b=1, h=12, w=16, s=3),     # F = 12: v1.0 scales 2-3
                                  dict(g=1, f=12, b=2, h=8, w=8, s=10)])
def test_lowpass_block_grad(irdu, term_path, case):
    """LocalLowpassFilteringBlock (v1 feature convs + two-scale solver + skip), every parameter."""
    torch.manual_seed(5)
    c = case["g"] * case["f"]
    blk = irdu.LocalLowpassFilteringBlock(dim=c, nsubnets=1, ngraphs=case["g"], n_cgd_iters=case["s"])
    perturb_mixture(blk.local_filter, 51)
    with torch.no_grad():
        blk.skip_weight.copy_(torch.tensor([0.4, 0.9]))
    x = rand(case["b"], c, case["h"], case["w"], seed=19)
    check(blk, lambda xd, p: O.lowpass_block(xd, p, case["g"]), x)


def test_msgf_grad(irdu):
    """MultiScaleGraphFilter with the v13 feature CNN, S = 10: LocalNonLinearBlocks (LNBFn),
    convs and solver all on their HIP forward + reverse kernels."""
    torch.manual_seed(6)
    m = irdu.MultiScaleGraphFilter(3, 3, ngraphs=4, n_cgd_iters=10)
    perturb_mixture(m.localfilter, 61)
    x = torch.rand(2, 3, 16, 24)
    check(m, lambda xd, p: O.multiscale_graph_filter(xd, p, 4), x)


def test_abstract_model_grad(irdu):
    """End-to-end v1.0 model: encoder / 4 filter blocks / decoder, every parameter."""
    torch.manual_seed(8)
    dims, ng = (8, 12, 16, 24), (2, 2, 4, 4)
    m = irdu.AbtractMultiScaleGraphFilter(3, 3, dims=dims, hidden_dims=(8, 12, 16, 24), ngraphs=ng,
                                          num_blocks=(1, 1, 1, 1), num_blocks_out=1, n_cgd_iters=3)
    for i in range(4):
        perturb_mixture(getattr(m, f"localfilter_scale_0{i}").local_filter, 70 + i)
    x = torch.rand(1, 3, 32, 32)
    # The filter inputs come from the encoder (fp32 GPU vs fp64 oracle, ~1e-6 apart), so an edge
    # whose |C x| sits within that distance of gamma can take the other soft-threshold branch
    # (REF:684-704 is discontinuous in d/dgamma there): gamma gradients get a loose bound here;
    # the lowpass tests above pin them at GTOL on identical inputs.
    check(m, lambda xd, p: O.abstract_forward(xd, p, ng, (1, 1, 1, 1), 1), x, tol=5e-4, loose=("gamma",))


@pytest.mark.parametrize("hw", [(10, 14), (12, 16)])      # 2x2/s2 data gradient: direct kernel / GEMM + interleave
@pytest.mark.parametrize("bkm", [(2, 12, 24), (1, 96, 192), (1, 24, 160)])
def test_conv_grads(irdu, bkm, hw):
    b, k, m = bkm
    from irdu_amd import solver_grad as SG
    x = rand(b, k, *hw, seed=3)
    w1 = rand(m, k, 1, 1, seed=4) * 0.2
    w2 = rand(m, k, 2, 2, seed=5) * 0.2
    for fn, ref, w in ((SG.Conv1x1Fn.apply, torch.nn.functional.conv2d, w1),
                       (SG.Conv2x2s2Fn.apply, lambda a, b_: torch.nn.functional.conv2d(a, b_, stride=2), w2)):
        xr, wr = x.clone().double().requires_grad_(True), w.clone().double().requires_grad_(True)
        out_r = ref(xr, wr)
        r = rand(*out_r.shape, seed=6).double()
        (out_r * r).sum().backward()
        xg, wg = x.to(DEV).requires_grad_(True), w.to(DEV).requires_grad_(True)
        (fn(xg, wg) * r.float().to(DEV)).sum().backward()
        assert rel_err(xg.grad, xr.grad) <= 1e-5
        assert rel_err(wg.grad, wr.grad) <= 1e-5


def test_training_step_reduces_loss(irdu):
    """A few Adam steps of the image filter on one noisy batch lower the L1 loss (the training
    loop of scripts_v2/...sigma25.py:139-232 on the HIP reverse)."""
    torch.manual_seed(9)
    m = irdu.MultiScaleGraphFilter(3, 3, ngraphs=4, n_cgd_iters=4).to(DEV)
    clean = torch.rand(4, 3, 32, 32, device=DEV)
    noisy = clean + 0.1 * torch.randn_like(clean)
    opt = torch.optim.Adam(m.parameters(), lr=2e-3)
    losses = []
    for _ in range(6):
        opt.zero_grad(set_to_none=True)
        loss = torch.nn.functional.l1_loss(m(noisy), clean)
        loss.backward()
        opt.step()
        losses.append(float(loss.detach()))
    assert all(torch.isfinite(torch.tensor(losses)))
    assert losses[-1] < losses[0]


@pytest.mark.parametrize("fused", [True, False])   # gate + depthwise reverse in one row pass / two kernels
@pytest.mark.parametrize("chw", [(12, 32, 16, 16), (96, 256, 20, 24), (33, 20, 9, 44), (160, 64, 8, 12),
                                 (8, 16, 6, 100), (8, 16, 5, 200), (8, 12, 4, 300)])
def test_local_nonlinear_block_grad(irdu, chw, fused):
    """LocalNonLinearBlock reverse on HIP (LN, W1, depthwise 3x3, gate, W2, skip) vs fp64 oracle;
    W = 100 / 200 run the fused gate-depthwise row kernel at V = 2 / 4, W = 300 the two kernels."""
    from irdu_amd import solver_grad as SG
    SG.FUSED_GATE_DW3 = fused
    c, hid, h, w = chw
    torch.manual_seed(31)
    blk = irdu.LocalNonLinearBlock(c, hid, 1)
    with torch.no_grad():
        blk.norm.weighted_transform.weight.mul_(1 + 0.2 * torch.randn_like(blk.norm.weighted_transform.weight))
        blk.skip_weight.copy_(torch.tensor([0.7, 1.3]))
    x = rand(2, c, h, w, seed=32)
    try:
        check(blk, lambda xd, p: O.local_nonlinear_block(xd, p, ""), x)
    finally:
        SG.FUSED_GATE_DW3 = True
