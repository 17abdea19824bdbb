"""Depthwise 3x3 (replicate padding) forward and reverse of the LocalNonLinearBlock training path
(grr_dwconv3, grr_dwconv3_bwd: row-streaming kernels for W <= 256, per-pixel kernels above)
against float64 PyTorch autograd of the same op (REF:946 `F.pad(mode="replicate")` + grouped conv)."""
import pytest
import torch

from tests.test_gpu_parity import DEV, rel_err

pytestmark = pytest.mark.gpu

# widths: 1 / 2 / 4 columns per lane (32, 100, 200, 256 with idle lanes at 100 and 200), and the
# per-pixel fallback (300, 258); short planes and segmented grids (few planes, many rows)
SHAPES = [(2, 6, 8, 32), (1, 4, 17, 100), (1, 3, 40, 200), (2, 5, 33, 256), (1, 2, 9, 300), (1, 2, 70, 258),
          (1, 1, 300, 64), (1, 2, 1, 64), (1, 2, 2, 128)]


def _ref(h, w):
    c = h.shape[1]
    return torch.nn.functional.conv2d(torch.nn.functional.pad(h, (1, 1, 1, 1), mode="replicate"),
                                      w.view(c, 1, 3, 3), groups=c)


@pytest.fixture(scope="module")
def K():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import irdu_amd
    irdu_amd.load_native()
    from irdu_amd import kernels
    return kernels


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "b{}c{}h{}w{}".format(*s))
def test_dwconv3_forward_and_reverse_vs_autograd(K, shape):
    b, c, hh, ww = shape
    torch.manual_seed(hh * 7 + ww)
    h = torch.randn(b, c, hh, ww, dtype=torch.float64)
    w = torch.randn(c, 9, dtype=torch.float64)
    g = torch.randn(b, c, hh, ww, dtype=torch.float64)
    hr, wr = h.clone().requires_grad_(True), w.clone().requires_grad_(True)
    out = _ref(hr, wr)
    out.backward(g)
    got = K.dwconv3(h.float().to(DEV), w.float().to(DEV))
    gw = torch.zeros(c, 9, device=DEV)
    gh = K.dwconv3_bwd(g.float().to(DEV), h.float().to(DEV), w.float().to(DEV), gw)
    torch.cuda.synchronize()
    assert rel_err(got.cpu(), out.detach()) <= 2e-6
    assert rel_err(gh.cpu(), hr.grad) <= 2e-6
    assert rel_err(gw.cpu(), wr.grad) <= 2e-5
