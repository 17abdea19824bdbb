"""grr_wgrad (the weight gradients of the feature CNN's convolutions and LNB GEMMs, REF:556-612 /
REF13:564-575 under autograd) against a float64 CPU reduction.  fp32 products and sums in a fixed
order: within fp32 rounding of the exact sum, normwise 1e-5 at these sizes (the reduction runs over up
to 2^19 pixels; fp32 summation error grows like sqrt(n) eps); bitwise repeatable; ragged pixel
counts, P % 4 != 0, row counts that are not multiples of the 128 x 96 tile."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module")
def K():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import irdu_amd
    irdu_amd.load_native()
    from irdu_amd import kernels
    return kernels


def _ref(a, b):
    a64, b64 = a.double().cpu(), b.double().cpu()
    bb, m = a64.shape[:2]
    k = b64.shape[1]
    return torch.einsum("bmp,bkp->mk", a64.reshape(bb, m, -1), b64.reshape(bb, k, -1))


@pytest.mark.parametrize("shape", [
    (2, 96, 192, 64, 64),      # conv1x1 96 -> 192 (features of the edge weights)
    (2, 512, 96, 32, 32),      # LNB gw1: 2 hid x C
    (2, 96, 256, 32, 48),      # LNB gw2: C x hid
    (1, 7, 5, 3, 5),           # tiny, P = 15 (P % 4 != 0, a single ragged step)
    (3, 130, 97, 17, 23),      # rows past the tiles, ragged chunks
    (1, 33, 200, 256, 256),    # one image, many chunks
    (4, 384, 12, 128, 128),    # 2x2-s2 conv of a 3-channel image (K = 4 x 3)
])
def test_wgrad_matches_float64(K, shape):
    b, m, k, h, w = shape
    g = torch.Generator().manual_seed(m * 31 + k)
    a = torch.randn(b, m, h, w, generator=g)
    x = torch.randn(b, k, h, w, generator=g)
    ref = _ref(a, x)
    got = K.wgrad(a.to(DEV), x.to(DEV))
    got2 = K.wgrad(a.to(DEV), x.to(DEV))
    torch.cuda.synchronize()
    assert torch.equal(got, got2), "grr_wgrad must be deterministic"
    err = float((got.double().cpu() - ref).abs().max() / ref.abs().max())
    assert err <= 1e-5, err


def test_wgrad_bench_shape_against_matmul(K):
    """The msgf training step's largest reduction (LNB gw1 at 16 x 256^2) against torch's fp32 GEMM."""
    torch.manual_seed(3)
    a = torch.randn(16, 512, 256, 256, device=DEV)
    x = torch.randn(16, 96, 256, 256, device=DEV)
    got = K.wgrad(a, x)
    ref = torch.matmul(a.reshape(16, 512, -1).double(), x.reshape(16, 96, -1).transpose(1, 2).double()).sum(0)
    err = float((got.double() - ref).abs().max() / ref.abs().max())
    assert err <= 1e-5, err


def test_conv_weight_gradients_match_autograd(K):
    """The training ops' weight gradients (1x1 and 2x2-s2 conv) equal float64 autograd of nn.Conv2d."""
    from irdu_amd import solver_grad as SG
    torch.manual_seed(4)
    x = torch.randn(2, 12, 20, 28, dtype=torch.float64)
    w1 = torch.randn(24, 12, 1, 1, dtype=torch.float64)
    w2 = torch.randn(16, 12, 2, 2, dtype=torch.float64)
    gy1 = torch.randn(2, 24, 20, 28, dtype=torch.float64)
    gy2 = torch.randn(2, 16, 10, 14, dtype=torch.float64)
    for w, gy, fn, conv in ((w1, gy1, SG.Conv1x1Fn, lambda x, w: torch.nn.functional.conv2d(x, w)),
                            (w2, gy2, SG.Conv2x2s2Fn, lambda x, w: torch.nn.functional.conv2d(x, w, stride=2))):
        wr = w.clone().requires_grad_(True)
        conv(x, wr).backward(gy)
        wd = w.float().to(DEV).requires_grad_(True)
        fn.apply(x.float().to(DEV).contiguous(), wd).backward(gy.float().to(DEV))
        err = float((wd.grad.double().cpu() - wr.grad).abs().max() / wr.grad.abs().max())
        assert err <= 1e-5, (fn, err)


@pytest.mark.parametrize("shape", [
    (2, 192, 48, 64, 64),      # v1.0 first-level W1 gradient: the 192 x 64 tile
    (2, 48, 192, 64, 64),      # ... transposed (the plan swaps the operands)
    (2, 48, 96, 64, 64),       # v1.0 first-level W2 gradient: the 64 x 96 tile, two waves per SIMD
    (1, 40, 70, 13, 11),       # 64 x 96 tile with rows past the tile, P % 4 != 0, ragged step
    (3, 170, 33, 9, 20),       # 192 x 64 tile with rows past it
    (1, 12, 7, 3, 3),          # tiny
])
@pytest.mark.parametrize("tiles", [True, False])
def test_wgrad_tile_plans_match_float64(K, shape, tiles):
    """Every wave tile the plan can take (grr_wgrad_set_tiles(1)) and the 128 x 96 tile alone (0), against
    the float64 reduction; each deterministic."""
    b, m, k, h, w = shape
    g = torch.Generator().manual_seed(m * 17 + k + h)
    a = torch.randn(b, m, h, w, generator=g)
    x = torch.randn(b, k, h, w, generator=g)
    ref = _ref(a, x)
    try:
        K.set_wgrad_tiles(tiles)
        got = K.wgrad(a.to(DEV), x.to(DEV))
        got2 = K.wgrad(a.to(DEV), x.to(DEV))
        torch.cuda.synchronize()
    finally:
        K.set_wgrad_tiles(True)
    assert torch.equal(got, got2)
    err = float((got.double().cpu() - ref).abs().max() / ref.abs().max())
    assert err <= 1e-5, err
