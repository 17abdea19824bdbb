"""The training reverse's elementwise / reduction glue kernels (grr_bwd_lincomb, grr_bwd_graph_dot,
grr_bwd_unpool2_acc; the adjoints of the per-graph scalings, the per-graph inner products and the
2x2 upsampling U of REF:676-679) against plain torch on the same tensors: the float4 paths (W % 4 == 0,
16-byte aligned) and the scalar paths (odd widths, offset views)."""
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


SHAPES = [(2, 4, 3, 16, 32), (1, 2, 3, 7, 9), (3, 5, 1, 10, 6), (16, 32, 3, 64, 64)]


def _per_graph(v, b, g, f):
    return v.view(1, g, 1, 1, 1).expand(b, g, f, 1, 1)


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "b{}g{}f{}h{}w{}".format(*s))
@pytest.mark.parametrize("acc", [False, True])
def test_lincomb(K, shape, acc):
    b, g, f, h, w = shape
    x = torch.randn(b, g * f, h, w, device=DEV)
    y = torch.randn_like(x)
    sa, sb = torch.randn(g, device=DEV), torch.randn(g, device=DEV)
    out0 = torch.randn_like(x)
    for use_y, use_sa, use_sb in ((True, True, True), (False, True, False), (True, False, True), (True, True, False)):
        ref = (_per_graph(sa, b, g, f) if use_sa else 1.0) * x.view(b, g, f, h, w)
        if use_y:
            ref = ref + (_per_graph(sb, b, g, f) if use_sb else 1.0) * y.view(b, g, f, h, w)
        ref = ref.reshape(b, g * f, h, w) + (out0 if acc else 0.0)
        out = out0.clone()
        K.bwd_lincomb(x, sa if use_sa else None, y if use_y else None, sb if use_sb else None, g, out=out,
                      accumulate=acc)
        torch.testing.assert_close(out, ref, rtol=1e-6, atol=1e-6)


def test_lincomb_unaligned_view(K):
    """A view one float into its storage: the scalar path."""
    base = torch.randn(2 * 6 * 8 * 8 + 1, device=DEV)
    x = base[1:].view(2, 6, 8, 8)
    sa = torch.randn(2, device=DEV)
    out = K.bwd_lincomb(x, sa, None, None, 2)
    ref = sa.view(1, 2, 1, 1, 1) * x.view(2, 2, 3, 8, 8)
    torch.testing.assert_close(out, ref.reshape(2, 6, 8, 8), rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "b{}g{}f{}h{}w{}".format(*s))
def test_graph_dot(K, shape):
    b, g, f, h, w = shape
    u = torch.randn(b, g * f, h, w, device=DEV)
    v = torch.randn_like(u)
    out = torch.full((g,), 0.5, device=DEV)
    K.bwd_graph_dot(u, v, out, g, coef=-1.5)
    ref = 0.5 - 1.5 * (u.double() * v.double()).view(b, g, -1).sum(dim=(0, 2))
    torch.testing.assert_close(out.double(), ref, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("shape", [(2, 3, 8, 16), (1, 2, 6, 10), (4, 96, 64, 256), (1, 1, 2, 2)])
def test_unpool2_acc(K, shape):
    b, c, h, w = shape
    xd = torch.randn(b, c, h // 2, w // 2, device=DEV)
    out0 = torch.randn(b, c, h, w, device=DEV)
    out = out0.clone()
    K.bwd_unpool2_acc(xd, out)
    ref = out0 + 0.25 * xd.repeat_interleave(2, dim=2).repeat_interleave(2, dim=3)
    torch.testing.assert_close(out, ref, rtol=1e-6, atol=1e-6)
