"""The fused LocalNonLinearBlock with its input and / or output in the channel-blocked layout
(grr_lnb_forward_c8, kernels.lnb_forward_c8): bitwise equal to the [B, C, H, W] pass -- the same arithmetic on
the same registers, only the memory instructions differ -- and the image filter's feature chains that pass
blocked tensors between blocks (graph_filter.run_blocks) equal the per-block path bitwise."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def K():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import irdu_amd
    irdu_amd.load_native()
    from irdu_amd import kernels
    return kernels


def _block(c, hid, seed):
    import irdu_amd
    torch.manual_seed(seed)
    blk = irdu_amd.LocalNonLinearBlock(c, hid, 1)
    with torch.no_grad():
        for p in blk.parameters():
            p.copy_(torch.randn_like(p) * (0.3 if p.dim() > 1 else 1.0))
        blk.skip_weight.copy_(torch.tensor([0.7, 1.3]))
    return blk.to(DEV).eval()


@pytest.mark.parametrize("c,hid,b,h,w", [(96, 256, 2, 40, 72), (96, 256, 1, 256, 256), (48, 96, 3, 17, 33),
                                         (6, 16, 2, 9, 31), (20, 40, 1, 8, 8), (96, 256, 4, 128, 128)])
def test_c8_layouts_bitwise(K, c, hid, b, h, w):
    blk = _block(c, hid, c + h)
    x = torch.randn(b, c, h, w, device=DEV) * 2.0
    with torch.no_grad():
        ref = blk(x)
        x8 = K.to_c8(x)
        assert x8.shape == (b, (c + 7) // 8, h, w, 8)
        assert torch.equal(K.from_c8(x8, c), x)
        if c % 8:
            assert torch.count_nonzero(x8[:, -1, :, :, c % 8:]) == 0          # pad channels 0
        for layout in range(4):
            xin = x8 if layout & 1 else x
            out = blk._forward_c8(xin, bool(layout & 1), bool(layout & 2))
            if layout & 2:
                if c % 8:
                    assert torch.count_nonzero(out[:, -1, :, :, c % 8:]) == 0  # pads written 0
                out = K.from_c8(out, c)
            assert torch.equal(out, ref), (layout, (out - ref).abs().max().item())


def test_feature_chain_blocked_equals_per_block(K):
    import irdu_amd
    from irdu_amd import graph_filter as GF
    from tests.test_gpu_parity import perturb_mixture
    torch.manual_seed(3)
    m = irdu_amd.MultiScaleGraphFilter(3, 3, ngraphs=32, n_cgd_iters=10)
    perturb_mixture(m.localfilter, 5)
    m = m.to(DEV).eval()
    img = torch.rand(2, 3, 64, 96, device=DEV)
    saved = GF.BLOCKED_CHAINS
    try:
        with torch.no_grad():
            GF.BLOCKED_CHAINS = False
            ref = m(img)
            GF.BLOCKED_CHAINS = True
            got = m(img)
    finally:
        GF.BLOCKED_CHAINS = saved
    assert torch.equal(got, ref), (got - ref).abs().max().item()
