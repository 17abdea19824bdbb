"""Depthwise 3x3 (replicate padding) forward and reverse of the LocalNonLinearBlock training path
(grr_dwconv3, grr_dwconv3_bwd: row-streaming kernels, column strips for W > 256, per-pixel kernels for
W > 128 with W % 4 != 0)
against float64 PyTorch autograd of the same op (REF:946 `F.pad(mode="replicate")` + grouped conv)."""
import pytest
import torch

from tests.test_gpu_parity import DEV, rel_err

pytestmark = pytest.mark.gpu

# widths: 1 / 2 / 4 columns per lane (32, 100, 200, 256 with idle lanes at 100 and 200), column strips
# of 248 owned columns for W > 256 with W % 4 == 0 (300, 512, 744 = 3 x 248, 1000), the per-pixel
# fallback (258); short planes and segmented grids (few planes, many rows)
SHAPES = [(2, 6, 8, 32), (1, 4, 17, 100), (1, 3, 40, 200), (2, 5, 33, 256), (1, 2, 9, 300), (1, 2, 70, 258),
          (1, 1, 300, 64), (1, 2, 1, 64), (1, 2, 2, 128), (1, 2, 12, 512), (1, 1, 7, 744), (2, 1, 5, 1000)]


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


def _gate_ref(hh, w, ffn):
    """(LNB) replicate-pad depthwise, sigmoid(m) m v  /  (FFN) zero-pad depthwise, gelu(m) v."""
    c2 = hh.shape[1]
    if ffn:
        d = torch.nn.functional.conv2d(hh, w.view(c2, 1, 3, 3), padding=1, groups=c2)
    else:
        d = _ref(hh, w)
    m, v = d.chunk(2, dim=1)
    return (torch.nn.functional.gelu(m) if ffn else torch.sigmoid(m) * m) * v


@pytest.mark.parametrize("ffn", [False, True], ids=["lnb", "ffn"])
@pytest.mark.parametrize("shape", [(2, 3, 9, 32), (1, 4, 20, 100), (1, 2, 33, 256), (1, 2, 10, 300), (1, 3, 12, 512),
                                   (1, 1, 6, 744)], ids=lambda s: "b{}hid{}h{}w{}".format(*s))
def test_gate_dw3_rows_vs_autograd(K, shape, ffn):
    """The fused depthwise + gate row kernels (forward: grr_lnb_dw3_gate / grr_ffn_dw3_gate; reverse with
    the depthwise output recomputed: grr_lnb_gate_dw3_bwd / grr_ffn_gate_dw3_bwd) against float64 autograd,
    including column strips (W > 256)."""
    b, hid, hh_, ww = shape
    torch.manual_seed(hh_ * 11 + ww + int(ffn))
    hh = torch.randn(b, 2 * hid, hh_, ww, dtype=torch.float64)
    w = torch.randn(2 * hid, 9, dtype=torch.float64) * 0.5
    gq = torch.randn(b, hid, hh_, ww, dtype=torch.float64)
    s = 0.7
    hr, wr = hh.clone().requires_grad_(True), w.clone().requires_grad_(True)
    gate = _gate_ref(hr, wr, ffn)
    (s * (gq * gate).sum()).backward()
    hd, wd = hh.float().to(DEV), w.float().to(DEV)
    got = (K.ffn_dw3_gate if ffn else K.lnb_dw3_gate)(hd, wd)
    gw = torch.zeros(2 * hid, 9, device=DEV)
    gdot = torch.zeros(1, device=DEV)
    sc = torch.tensor([s], device=DEV)
    if ffn:
        gh = K.ffn_gate_dw3_bwd(gq.float().to(DEV), sc, hd, wd, gw, gdot)
    else:
        gh = K.lnb_gate_dw3_bwd(None, gq.float().to(DEV), sc, hd, wd, gw, gdot)
    torch.cuda.synchronize()
    assert rel_err(got.cpu(), gate.detach()) <= 2e-6
    assert rel_err(gh.cpu(), hr.grad) <= 2e-5
    assert rel_err(gw.cpu(), wr.grad) <= 2e-5
    assert abs(float(gdot) - float((gq * gate).sum())) <= 2e-5 * float((gq * gate).abs().sum())


RING_SHAPES = [(2, 3, 9, 32), (1, 4, 20, 100), (1, 2, 33, 256), (1, 2, 10, 300), (1, 3, 12, 512), (1, 1, 6, 744),
               (1, 2, 300, 64), (1, 2, 1, 64), (1, 2, 2, 128), (2, 1, 5, 1000), (1, 5, 40, 200), (1, 2, 7, 102),
               (1, 2, 9, 264), (2, 3, 70, 512)]   # the one-strip V = 8 instance: 33 of 64 lanes, a whole row


@pytest.mark.parametrize("shape", RING_SHAPES, ids=lambda s: "b{}hid{}h{}w{}".format(*s))
def test_gate_dw3_bwd_ring_equals_register_kernel(K, shape):
    """grr_lnb_gate_dw3_bwd's per-wave LDS-ring kernel (default) against the register row kernel: the same
    expressions in the same order (gh to fp32 contraction, the weight-gradient and <gq, gate> reductions to
    summation order); segmented grids (300 rows), 1- and 2-row images, strips (W > 256), W % 4 != 0 (the ring
    declines: the register kernel runs both)."""
    b, hid, hh_, ww = shape
    torch.manual_seed(hh_ * 13 + ww)
    hh = torch.randn(b, 2 * hid, hh_, ww, device=DEV)
    w = torch.randn(2 * hid, 9, device=DEV) * 0.5
    gq = torch.randn(b, hid, hh_, ww, device=DEV)
    sc = torch.tensor([0.7], device=DEV)
    res = {}
    try:
        for ring in (False, True):
            K.set_lnb_bwd_ring(ring)
            gw = torch.zeros(2 * hid, 9, device=DEV)
            gdot = torch.zeros(1, device=DEV)
            gh = K.lnb_gate_dw3_bwd(None, gq, sc, hh, w, gw, gdot)
            torch.cuda.synchronize()
            res[ring] = (gh.cpu(), gw.cpu(), gdot.cpu())
    finally:
        K.set_lnb_bwd_ring(True)
    (g1, w1, d1), (g0, w0, d0) = res[True], res[False]
    assert torch.isfinite(g1).all()
    assert rel_err(g1, g0) <= 2e-6, rel_err(g1, g0)
    assert rel_err(w1, w0) <= 1e-5, rel_err(w1, w0)
    assert abs(float(d1) - float(d0)) <= 1e-5 * max(1.0, abs(float(d0))) * (b * hid * hh_ * ww) ** 0.5
