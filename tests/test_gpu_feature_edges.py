"""The feature 1x1 conv + edge weights in one pass (grr_feature_edges, kernels.feature_edges) against the two-pass
path (conv1x1 then edge_weights_block) and against a float64 restatement of REF:146-175 on the same features,
at strip edges (29-column strips), row segments, partial graph tiles (G < 32) and both input layouts."""
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


def _edges64(feat, mm):
    """float64 extract_edge_weights of one slab: feat [B, G, 3, H, W], mm [G, 3] -> w [B, G, 4, H, W] (up, left,
    right, down; replicate neighbours), pair weights [B, G, 2, H, W]."""
    n = feat / feat.norm(dim=2, keepdim=True).clamp_min(1e-12) * mm[None, :, :, None, None]
    up = torch.cat([n[..., :1, :], n[..., :-1, :]], -2)
    dn = torch.cat([n[..., 1:, :], n[..., -1:, :]], -2)
    lf = torch.cat([n[..., :1], n[..., :-1]], -1)
    rt = torch.cat([n[..., 1:], n[..., -1:]], -1)
    s = torch.stack([(n * up).sum(2), (n * lf).sum(2), (n * rt).sum(2), (n * dn).sum(2)], 2)
    w = torch.softmax(s, 2)
    ch = w[:, :, 2] ** 2
    ch[..., :-1] = ch[..., :-1] + w[:, :, 1, :, 1:] ** 2
    ch[..., -1] = 0
    cv = w[:, :, 3] ** 2
    cv[..., :-1, :] = cv[..., :-1, :] + w[:, :, 0, 1:, :] ** 2
    cv[..., -1, :] = 0
    return w, torch.stack([ch, cv], 2)


@pytest.mark.parametrize("b,g,h,w", [(2, 32, 40, 64), (1, 32, 256, 256), (2, 5, 9, 29), (1, 13, 33, 30),
                                     (3, 32, 8, 59), (1, 32, 70, 100), (2, 8, 1, 31), (1, 32, 128, 128)])
def test_feature_edges_vs_two_pass_and_float64(K, b, g, h, w):
    c = 3 * g
    torch.manual_seed(b * 100 + g + h + w)
    x = (torch.randn(b, c, h, w) * torch.rand(b, 1, h, w) * 3).to(DEV)   # per-pixel scales vary
    wt = (torch.randn(2 * c, c, 1, 1) * 0.2).to(DEV)
    mG = (0.5 + torch.rand(g, 3)).to(DEV)
    mL = (0.5 + torch.rand(g, 3)).to(DEV)
    wG, cG, wL = K.feature_edges(x, False, wt, g, 3, mG, mL)
    feat = K.conv1x1(x, wt)
    rG, rc, rL = K.edge_weights_block(feat, g, 3, mG, mL)
    for got, ref in ((wG, rG), (cG, rc), (wL, rL)):
        assert torch.allclose(got, ref, rtol=1e-4, atol=1e-5), (got - ref).abs().max().item()
    f64 = torch.nn.functional.conv2d(x.double().cpu(), wt.double().cpu())
    for slab, (got_w, mm) in enumerate(((wG, mG), (wL, mL))):
        fr = f64[:, slab * c:(slab + 1) * c].reshape(b, g, 3, h, w)
        w64, c64 = _edges64(fr, mm.double().cpu())
        assert (got_w.double().cpu() - w64).abs().max().item() < 2e-5, slab
        if slab == 0:
            assert (cG.double().cpu() - c64).abs().max().item() < 4e-5
    # the channel-blocked input is the same arithmetic
    wG8, cG8, wL8 = K.feature_edges(K.to_c8(x), True, wt, g, 3, mG, mL)
    assert torch.equal(wG8, wG) and torch.equal(cG8, cG) and torch.equal(wL8, wL)


def test_image_filter_fused_edges_close_to_two_pass(K):
    import irdu_amd
    from irdu_amd import graph_filter as GF
    from tests.test_gpu_parity import perturb_mixture
    torch.manual_seed(5)
    m = irdu_amd.MultiScaleGraphFilter(3, 3, ngraphs=32, n_cgd_iters=10)
    perturb_mixture(m.localfilter, 9)
    m = m.to(DEV).eval()
    img = torch.rand(2, 3, 96, 128, device=DEV)
    saved = GF.FUSED_FEATURE_EDGES
    try:
        with torch.no_grad():
            GF.FUSED_FEATURE_EDGES = False
            ref = m(img)
            GF.FUSED_FEATURE_EDGES = True
            got = m(img)
    finally:
        GF.FUSED_FEATURE_EDGES = saved
    err = (got - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-5, err
