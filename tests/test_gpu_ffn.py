"""grr_ffn_forward: the window models' FFBlock (REF7:13-67: CustomLayerNorm, 1x1 -> depthwise 3x3 with
zero padding -> exact-erf gelu gate -> 1x1, weighted skip) against the module's own PyTorch ops in
float64 on the CPU.  The GEMMs use the exact 3-term bf16 split (six products), so the HIP block must be
as accurate as a plain fp32 evaluation of the same ops (4x the fp32 CPU error against float64, as in
test_x3_gemm_is_fp32_accurate) and within the 1e-4 relative contract.  Shapes: the K <= 128 GEMM path
with in-kernel LN statistics (C = 48, 128) and the K-streaming path with the ln_stats scale (C = 256),
hidden widths that are not multiples of the 32-row tiles, odd image sizes (zero-padding frame)."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module")
def W():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import irdu_amd
    irdu_amd.load_native()
    from irdu_amd import window_graph
    return window_graph


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / b.abs().max())


def _block(W, c, seed):
    torch.manual_seed(seed)
    blk = W.FFBlock(c, 2.6666, False)
    with torch.no_grad():   # move the weights off their init so every part of the block matters
        blk.norm.weighted_transform.weight.uniform_(0.5, 1.5)
        blk.skip_connect_weight_final.copy_(torch.tensor([0.7, 1.3]))
    return blk


@pytest.mark.parametrize("shape", [(2, 48, 17, 23), (2, 128, 64, 64), (1, 256, 32, 48), (1, 130, 9, 70)])
def test_ffblock_matches_float64(W, shape):
    b, c, h, w = shape
    blk = _block(W, c, seed=c + h)
    x = torch.randn(b, c, h, w, generator=torch.Generator().manual_seed(7)) * 2.0 + 0.3
    with torch.no_grad():
        ref64 = copy.deepcopy(blk).double()(x.double())
        ref32 = blk(x)
        got = copy.deepcopy(blk).to(DEV)(x.to(DEV))
    err32 = _rel(ref32, ref64)
    err = _rel(got, ref64)
    assert err <= 4 * err32 + 1e-7, (err, err32)
    assert err <= 1e-4


def test_feature_extraction_matches_cpu(W):
    """The whole window feature CNN (FFBlocks on HIP, 3x3 convs on stock ops) against the CPU module."""
    torch.manual_seed(3)
    fe = W.FeatureExtraction(inp_channels=3, out_channels=40, dim=32, num_blocks=[2, 1, 1], num_refinement_blocks=1,
                             ffn_expansion_factor=2.6666, bias=False)
    x = torch.rand(2, 3, 32, 40)
    with torch.no_grad():
        ref = fe(x)[0]
        got = copy.deepcopy(fe).to(DEV)(x.to(DEV))[0]
    assert _rel(got, ref) <= 1e-4


@pytest.mark.parametrize("shape", [(2, 32, 16, 24), (1, 128, 33, 64), (1, 48, 20, 128), (1, 64, 12, 256)])
def test_ffblock_gradients_match_float64(W, shape):
    """Training path (solver_grad.FFNFn: HIP forward, HIP reverse with the zero-pad / gelu row kernels)
    against float64 autograd of the module's PyTorch ops on the CPU: the input and every parameter
    (CustomLayerNorm scale, W_in, depthwise taps, W_out, skip weights).  Row widths V = 1 / 2 / 4."""
    b, c, h, w = shape
    blk = _block(W, c, seed=c + w)
    x = torch.randn(b, c, h, w, generator=torch.Generator().manual_seed(9))
    gout = torch.randn(b, c, h, w, generator=torch.Generator().manual_seed(10))
    ref = copy.deepcopy(blk).double()
    xr = x.double().requires_grad_(True)
    ref(xr).backward(gout.double())
    dev = copy.deepcopy(blk).to(DEV)
    xd = x.to(DEV).requires_grad_(True)
    out = dev(xd)
    out.backward(gout.to(DEV))
    assert _rel(xd.grad, xr.grad) <= 1e-4, "x"
    for (k, pr), (_, pd) in zip(ref.named_parameters(), dev.named_parameters()):
        assert _rel(pd.grad, pr.grad) <= 1e-4, k


def test_ffblock_training_uses_hip(W):
    """The recorded graph of a CUDA FFBlock is the opaque HIP op, not the stock conv ops."""
    blk = _block(W, 32, seed=1).to(DEV)
    x = torch.randn(1, 32, 8, 8, device=DEV, requires_grad=True)
    out = blk(x)
    names = []
    fn = out.grad_fn
    while fn is not None and len(names) < 8:
        names.append(type(fn).__name__)
        fn = fn.next_functions[0][0] if fn.next_functions else None
    assert not any("Convolution" in n for n in names), names
    out.sum().backward()
    assert x.grad is not None and blk.ffn.project_in.weight.grad is not None
