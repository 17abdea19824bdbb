"""Gradients of the GLRFast / GTVFast module methods (the reference differentiates these ATen
compositions with autograd, REF = exploration/GGTV_GGLR_v1.0/deep_multiscale_GGLR_GGTV_v1x0.py
:128-228, :452-516): the HIP reverses (csrc/subapi_bwd.hip through solver_grad's opaque functions)
against float64 autograd through the oracle's restatement of the same methods, on odd image sizes
so every replicate / zero / frame-drop boundary rule is exercised.  Tolerance: max-abs error over
max-abs reference gradient <= 2e-5 (fp32 kernels vs fp64 reference)."""
import pytest
import torch

from oracle import graph_oracle as O
from tests.test_gpu_parity import DEV, perturbed_graph_module, rand

pytestmark = pytest.mark.gpu

B, G, F, H, W = 2, 3, 4, 9, 13


@pytest.fixture(scope="module")
def irdu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import irdu_amd
    irdu_amd.load_native()
    return irdu_amd


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _module(irdu, cls, seed):
    torch.manual_seed(seed)
    m = getattr(irdu, cls)(F, G, 1.0)
    perturbed_graph_module(m, seed + 1)
    return m


def _ref_params(m):
    """The module's parameters as float64 leaves keyed like the oracle's parameter dicts."""
    return {k: v.detach().cpu().double().clone().requires_grad_(True) for k, v in m.state_dict().items()}


def _hip_grads(m, fn, inputs, gout):
    ins = [t.to(DEV).requires_grad_(True) for t in inputs]
    m = m.to(DEV)
    for p in m.parameters():
        p.grad = None
    out = fn(m, *ins)
    out.backward(gout.to(DEV))
    return out, [t.grad for t in ins], {k: p.grad for k, p in m.named_parameters() if p.grad is not None}


def _check(out, ref_out, gin, ref_in, gp, ref_p, tol=2e-5):
    assert rel(out, ref_out) <= 1e-5
    for a, b in zip(gin, ref_in):
        assert rel(a, b) <= tol
    for k, g in gp.items():
        assert rel(g, ref_p[k].grad) <= tol, k


def test_get_neighbors_pixels_grad(irdu):
    m = _module(irdu, "GLRFast", 1)
    x = rand(B, G * F, H, W, seed=2)
    gout = rand(B, G * F, 4, H, W, seed=3)
    out, gin, _ = _hip_grads(m, lambda mm, a: mm.get_neighbors_pixels(a), [x], gout)
    xr = x.double().requires_grad_(True)
    ref = O.gather_neighbors(xr)
    ref.backward(gout.double())
    _check(out, ref, gin, [xr.grad], {}, {})


def test_normalize_and_transform_features_grad(irdu):
    m = _module(irdu, "GLRFast", 4)
    f5 = rand(B, G, F, H, W, seed=5)
    with torch.no_grad():
        f5[0, 1, :, 2, 3] = 0.0                      # a zero feature vector (|f| below eps)
    gout = rand(B, G * F, H, W, seed=6)
    out, gin, gp = _hip_grads(m, lambda mm, a: mm.normalize_and_transform_features(a), [f5], gout)
    p = _ref_params(m)
    fr = f5.double().requires_grad_(True)
    ref = O.normalize_features(fr, p["multiM"])
    ref.backward(gout.double())
    _check(out, ref, gin, [fr.grad], gp, p)


@pytest.mark.parametrize("transpose", [False, True])
def test_stats_conv_grad(irdu, transpose):
    m = _module(irdu, "GTVFast", 7)
    x5 = rand(B, G, F, H, W, seed=8)
    gout = rand(B, G, F, H, W, seed=9)
    fn = (lambda mm, a: mm.stats_conv_transpose(a)) if transpose else (lambda mm, a: mm.stats_conv(a))
    out, gin, gp = _hip_grads(m, fn, [x5], gout)
    p = _ref_params(m)
    xr = x5.double().requires_grad_(True)
    k = O.stats_kernel(p, "")
    ref = O.stats_conv_t(xr, k) if transpose else O.stats_conv(xr, k)
    ref.backward(gout.double())
    _check(out, ref, gin, [xr.grad], gp, p)


def _weights(seed):
    return torch.softmax(rand(B, G, 4, H, W, seed=seed, scale=2.0), dim=2)


def test_op_L_norm_grad(irdu):
    m = _module(irdu, "GLRFast", 10)
    x5, w = rand(B, G, F, H, W, seed=11), _weights(12)
    gout = rand(B, G, F, H, W, seed=13)
    out, gin, _ = _hip_grads(m, lambda mm, a, b: mm.op_L_norm(a, b), [x5, w], gout)
    xr, wr = x5.double().requires_grad_(True), w.double().requires_grad_(True)
    nb = O.gather_neighbors(xr.reshape(B, G * F, H, W)).view(B, G, F, 4, H, W)
    ref = xr - torch.einsum("bgfehw,bgehw->bgfhw", nb, wr)    # REF:222-226
    ref.backward(gout.double())
    _check(out, ref, gin, [xr.grad, wr.grad], {}, {})


def test_op_C_grad(irdu):
    m = _module(irdu, "GTVFast", 14)
    x5, w = rand(B, G, F, H, W, seed=15), _weights(16)
    gout = rand(B, G, F, 4, H, W, seed=17)
    out, gin, gp = _hip_grads(m, lambda mm, a, b: mm.op_C(a, b), [x5, w], gout)
    p = _ref_params(m)
    xr, wr = x5.double().requires_grad_(True), w.double().requires_grad_(True)
    ref = O.gtv_C(xr, wr, O.stats_kernel(p, ""))
    ref.backward(gout.double())
    _check(out, ref, gin, [xr.grad, wr.grad], gp, p)


def test_op_C_transpose_grad(irdu):
    m = _module(irdu, "GTVFast", 18)
    e6, w = rand(B, G, F, 4, H, W, seed=19), _weights(20)
    gout = rand(B, G, F, H, W, seed=21)
    out, gin, gp = _hip_grads(m, lambda mm, a, b: mm.op_C_transpose(a, b), [e6, w], gout)
    p = _ref_params(m)
    er, wr = e6.double().requires_grad_(True), w.double().requires_grad_(True)
    ref = O.gtv_Ct(er, wr, O.stats_kernel(p, ""))
    ref.backward(gout.double())
    _check(out, ref, gin, [er.grad, wr.grad], gp, p)


def test_sub_api_composition_matches_forward_grads(irdu):
    """The reference composes the methods into GTVFast.forward = op_C_transpose(op_C(x)) (REF:518-523):
    differentiating the composition equals differentiating the fused forward."""
    m = _module(irdu, "GTVFast", 22).to(DEV)
    x5, w = rand(B, G, F, H, W, seed=23).to(DEV), _weights(24).to(DEV)
    gout = rand(B, G, F, H, W, seed=25).to(DEV)
    grads = []
    for fn in (lambda a, b: m.op_C_transpose(m.op_C(a, b), b), lambda a, b: m(a, b)):
        xa, wa = x5.clone().requires_grad_(True), w.clone().requires_grad_(True)
        for p in m.parameters():
            p.grad = None
        fn(xa, wa).backward(gout)
        grads.append([xa.grad, wa.grad] + [p.grad for p in m.parameters() if p.grad is not None])
    for a, b in zip(*grads):
        assert rel(a, b) <= 2e-5
