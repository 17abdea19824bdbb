"""GPU parity: the HIP path (libgrr.so through irdu_amd) against the CPU oracle.

Tolerance (north_star): fp32 outputs within 1e-4 relative, measured normwise as
max|hip - oracle| / max|oracle| over the tensor; the neighbour table is bit-exact;
PSNR within 0.01 dB.  Inputs are seeded; the oracle is pinned to the reference by
tests/test_oracle_golden.py, and the golden fixtures are also compared directly.
"""
import numpy as np
import pytest
import torch

from oracle import graph_oracle as O
from tests.golden_io import load_golden, params_of

pytestmark = pytest.mark.gpu

RTOL = 1e-4


@pytest.fixture(scope="module")
def irdu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import irdu_amd
    irdu_amd.load_native()
    return irdu_amd


DEV = "cuda"


@pytest.fixture(params=["auto", "strips", "independent"])
def variant(irdu, request):
    """Run a test with the row-wave graph kernels (auto, W <= 256) and with the column-strip
    kernels forced at every width."""
    irdu.kernels.set_kernel_variant(request.param)
    yield request.param
    irdu.kernels.set_kernel_variant("auto")


def rel_err(a, b):
    a = a.detach().double().cpu()
    b = torch.as_tensor(b).double().cpu()
    assert a.shape == b.shape, (a.shape, b.shape)
    return float((a - b).abs().max()) / max(float(b.abs().max()), 1e-30)


def assert_close(a, b, rtol=RTOL):
    e = rel_err(a, b)
    assert e <= rtol, f"relative error {e:.3e} > {rtol:.1e}"


def rand(*shape, seed=0, scale=1.0, offset=0.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g) * scale + offset


def perturbed_graph_module(mod, seed):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for p in (mod.stats_kernel_p01, mod.stats_kernel_p02a, mod.stats_kernel_p02b, mod.stats_kernel_p03):
            p.mul_(1 + 0.25 * torch.randn(p.shape, generator=g))
        mod.multiM.copy_(1 + 0.3 * torch.randn(mod.multiM.shape, generator=g))
    return mod


def perturb_mixture(mix, seed):
    g = torch.Generator().manual_seed(seed)
    u = lambda shape, lo, hi: lo + (hi - lo) * torch.rand(shape, generator=g)  # noqa: E731
    with torch.no_grad():
        mix.alphaCGD.copy_(u(mix.alphaCGD.shape, 0.2, 0.8))
        mix.betaCGD.copy_(u(mix.betaCGD.shape, 0.05, 0.4))
        for p in (mix.muys00, mix.muys01, mix.ro00, mix.ro01):
            p.copy_(torch.log(u(p.shape, 0.05, 0.6)))
        for p in (mix.gamma00, mix.gamma01):
            p.copy_(torch.log(u(p.shape, 0.002, 0.05)))
        for i, m in enumerate((mix.GLRmodule00, mix.GLRmodule01, mix.GTVmodule00, mix.GTVmodule01)):
            perturbed_graph_module(m, seed + 10 + i)


def sd_cpu(module):
    return {k: v.detach().cpu() for k, v in module.state_dict().items()}


# ---------------------------------------------------------------------------
# a1/a2: neighbour table, bit-exact
@pytest.mark.parametrize("hw", [(1, 1), (1, 7), (5, 1), (16, 20), (37, 45), (256, 256)])
def test_neighbor_table_bit_exact(irdu, hw):
    h, w = hw
    got = irdu.kernels.neighbor_table(h, w, DEV).cpu()
    assert torch.equal(got, O.neighbor_table(h, w))


def test_neighbor_table_matches_golden(irdu):
    d = load_golden("ops_small.npz")
    h, w = d["out/neighbor_table"].shape[-2:]
    assert np.array_equal(irdu.kernels.neighbor_table(h, w, DEV).cpu().numpy(), d["out/neighbor_table"])


# ---------------------------------------------------------------------------
# a3/a4 edge weights; a5-a10 operators — against the reference's golden vectors
def test_ops_golden(irdu):
    d = load_golden("ops_small.npz")
    feat = torch.from_numpy(d["in/feat"])
    x = torch.from_numpy(d["in/x"])
    b, g, f, h, w = x.shape
    glr = irdu.GLRFast(f, g, 1.0)
    gtv = irdu.GTVFast(f, g, 1.0)
    glr.load_state_dict(params_of(d, "glr."))
    gtv.load_state_dict(params_of(d, "gtv."))
    glr, gtv = glr.to(DEV), gtv.to(DEV)
    with torch.no_grad():
        wl, dl = glr.extract_edge_weights(feat.to(DEV))
        wg, dg = gtv.extract_edge_weights(feat.to(DEV))
        assert_close(wl, d["out/glr_w"], 1e-5)
        assert_close(dl, d["out/glr_deg"], 1e-5)
        assert_close(wg, d["out/gtv_w"], 1e-5)
        assert_close(glr(x.to(DEV), wl, dl), d["out/glr_forward"])
        assert_close(gtv(x.to(DEV), wg, dg), d["out/gtv_forward"])


@pytest.mark.parametrize("shape", [(2, 4, 3, 32, 32), (1, 2, 6, 37, 45), (2, 3, 12, 20, 70), (1, 2, 1, 64, 96)])
def test_edge_weights_random(irdu, shape):
    b, g, f, h, w = shape
    feat = rand(b, g, f, h, w, seed=1)
    m = perturbed_graph_module(irdu.GLRFast(f, g, 1.0), 3)
    wt, deg = m.to(DEV).extract_edge_weights(feat.to(DEV))
    ow, od = O.edge_weights(feat, m.multiM.detach().cpu())
    assert_close(wt, ow, 1e-5)
    assert_close(deg, od, 1e-5)


@pytest.mark.parametrize("shape", [(2, 4, 3, 32, 32), (1, 2, 6, 20, 64), (2, 3, 12, 9, 256), (1, 2, 1, 7, 40),
                                   (1, 2, 5, 12, 48), (1, 2, 3, 10, 300)])
def test_edge_weights_block(irdu, variant, shape):
    """The fused two-module edge weights (row-wave kernel for W <= 256 and F in {1,2,3,4,6,8,12,16},
    tile kernels otherwise) equal the per-module kernels + pair weights, and the oracle."""
    b, g, f, h, w = shape
    feat = rand(b, 2 * g * f, h, w, seed=41).to(DEV)
    mG, mL = ((1 + 0.3 * rand(g, f, seed=s)).to(DEV) for s in (42, 43))
    wG, cG, wL = irdu.kernels.edge_weights_block(feat, g, f, mG, mL)
    rG, _ = irdu.kernels.edge_weights(feat, 0, g, f, mG)
    rL, _ = irdu.kernels.edge_weights(feat, g * f, g, f, mL)
    assert_close(wG, rG, 1e-6)
    assert_close(wL, rL, 1e-6)
    assert_close(cG, irdu.kernels.gtv_pair_weights(rG), 1e-6)
    fo = feat.cpu().reshape(b, 2, g, f, h, w)
    assert_close(wG, O.edge_weights(fo[:, 0], mG.cpu())[0], 1e-5)
    assert_close(wL, O.edge_weights(fo[:, 1], mL.cpu())[0], 1e-5)


# widths: <= 64 (1 column per lane), 70 (2), 200 / 256 (4), 130 (W % 4 != 0 -> strips),
# 300 / 512 / 1000 (4 columns per lane in 248-column strips with 4 halo columns)
@pytest.mark.parametrize("shape", [(2, 4, 3, 32, 32), (1, 2, 6, 37, 45), (1, 3, 2, 9, 70), (1, 2, 3, 12, 200),
                                   (1, 1, 3, 10, 256), (1, 2, 3, 7, 130), (1, 1, 3, 11, 300), (1, 2, 3, 9, 512),
                                   (1, 1, 2, 6, 1000)])
def test_glr_gtv_operators_random(irdu, variant, shape):
    b, g, f, h, w = shape
    x = rand(b, g, f, h, w, seed=2)
    wl = torch.softmax(rand(b, g, 4, h, w, seed=3), dim=2)
    wg = torch.softmax(rand(b, g, 4, h, w, seed=4), dim=2)
    glr = perturbed_graph_module(irdu.GLRFast(f, g, 1.0), 5)
    gtv = perturbed_graph_module(irdu.GTVFast(f, g, 1.0), 6)
    kl = O.stats_kernel(sd_cpu(glr), "")
    kg = O.stats_kernel(sd_cpu(gtv), "")
    glr, gtv = glr.to(DEV), gtv.to(DEV)
    with torch.no_grad():
        assert_close(glr(x.to(DEV), wl.to(DEV)), O.glr_apply(x, wl, kl))
        assert_close(gtv(x.to(DEV), wg.to(DEV)), O.gtv_apply(x, wg, kg))


@pytest.mark.parametrize("shape", [(2, 4, 3, 32, 32), (1, 2, 6, 21, 31), (1, 2, 3, 10, 100), (1, 2, 3, 13, 132),
                                   (1, 2, 3, 8, 520)])
def test_gtv_prox_rhs_half(irdu, variant, shape):
    """C^T phi(C x) with the soft-threshold phi of the proximal step (a12, a16)."""
    b, g, f, h, w = shape
    x = rand(b, g, f, h, w, seed=7)
    wg = torch.softmax(rand(b, g, 4, h, w, seed=8), dim=2)
    gtv = perturbed_graph_module(irdu.GTVFast(f, g, 1.0), 9)
    kg = O.stats_kernel(sd_cpu(gtv), "")
    log_gamma = torch.log(torch.linspace(0.01, 0.2, g))
    t = O.gtv_C(x, wg, kg)
    e = O.soft_threshold(t, torch.exp(log_gamma))
    ref = O.gtv_Ct(e - (t - e), wg, kg)
    gtv = gtv.to(DEV)
    got = irdu.kernels.gtv_rhs_half(x.reshape(b, g * f, h, w).to(DEV), wg.to(DEV), irdu.kernels.stencil(gtv),
                                    True, log_gamma.to(DEV), g)
    assert_close(got.view(b, g, f, h, w), ref)
    # enough entries are thresholded for the test to mean something
    assert 0.05 < float((e == 0).double().mean()) < 0.95


# ---------------------------------------------------------------------------
# feature CNN
# K <= 128: split-bf16 MFMA path with the K column in registers; K > 128: the K-streaming split-bf16
# kernel (1 to 4 row tiles per workgroup, M tiles, odd K); the fp32 MFMA kernel (grr_conv1x1) directly
@pytest.mark.parametrize("bkmp", [(2, 12, 24, (8, 8)), (1, 96, 192, (33, 40)), (2, 7, 3, (5, 6)),
                                  (1, 96, 3, (16, 24)), (1, 160, 40, (9, 10)), (2, 512, 96, (16, 20)),
                                  (1, 200, 130, (7, 9)), (1, 384, 300, (12, 12)), (1, 129, 33, (5, 66)),
                                  (1, 256, 96, (3, 5))])
def test_conv1x1(irdu, bkmp):
    b, k, m, (h, w) = bkmp
    x = rand(b, k, h, w, seed=11)
    wt = rand(m, k, 1, 1, seed=12) * 0.2
    assert_close(irdu.kernels.conv1x1(x.to(DEV), wt.to(DEV)), torch.nn.functional.conv2d(x, wt), 1e-5)


def test_conv1x1_fp32_kernel(irdu):
    """grr_conv1x1 (fp32 MFMA, the ABI's plain entry point) at a deep K."""
    x = rand(1, 160, 9, 10, seed=11)
    wt = rand(40, 160, 1, 1, seed=12) * 0.2
    xd, wd = x.to(DEV), wt.to(DEV).contiguous()
    out = torch.empty(1, 40, 9, 10, device=DEV)
    from irdu_amd._native import call
    call("grr_conv1x1", xd.data_ptr(), wd.data_ptr(), out.data_ptr(), 1, 160, 40, 90,
         torch.cuda.current_stream().cuda_stream)
    assert_close(out, torch.nn.functional.conv2d(x, wt), 1e-5)


def test_x3_gemm_deep_k_is_fp32_accurate(irdu):
    """The K-streaming split-bf16 GEMM (K = 512, the LNB reverse's W1^T gh) against float64."""
    x = rand(2, 512, 20, 24, seed=34, scale=3.0, offset=0.5)
    wt = rand(96, 512, 1, 1, seed=35) * 0.1
    ref64 = torch.nn.functional.conv2d(x.double(), wt.double())
    err32 = rel_err(torch.nn.functional.conv2d(x, wt), ref64)
    err = rel_err(irdu.kernels.conv1x1(x.to(DEV), wt.to(DEV)), ref64)
    assert err <= 4 * err32 + 1e-7, (err, err32)


def test_x3_gemm_is_fp32_accurate(irdu):
    """The split-bf16 GEMM (3 exact bf16 terms per operand, 6 products) against a float64
    reference: its error must be of the order of a plain fp32 evaluation's, not bf16's."""
    x = rand(2, 96, 40, 36, seed=31, scale=3.0, offset=0.5)
    wt = rand(192, 96, 1, 1, seed=32) * 0.2
    ref64 = torch.nn.functional.conv2d(x.double(), wt.double())
    err32 = rel_err(torch.nn.functional.conv2d(x, wt), ref64)
    got = irdu.kernels.conv1x1(x.to(DEV), wt.to(DEV))
    err = rel_err(got, ref64)
    assert err <= 4 * err32 + 1e-7, (err, err32)
    # and the LayerNorm-folded variant inside the LNB (fp32 CPU oracle vs float64 oracle)
    torch.manual_seed(5)
    blk = irdu.LocalNonLinearBlock(96, 256, 1)
    p64 = {k: v.double() for k, v in sd_cpu(blk).items()}
    x = rand(1, 96, 24, 40, seed=33)
    ref64 = O.local_nonlinear_block(x.double(), p64, "")
    err32 = rel_err(O.local_nonlinear_block(x, sd_cpu(blk), ""), ref64)
    with torch.no_grad():
        err = rel_err(blk.to(DEV)(x.to(DEV)), ref64)
    assert err <= 4 * err32 + 1e-7, (err, err32)


@pytest.mark.parametrize("bkmhw", [(2, 12, 12, 16, 16), (1, 96, 96, 34, 50)])
def test_conv2x2s2(irdu, bkmhw):
    b, k, m, h, w = bkmhw
    x = rand(b, k, h, w, seed=13)
    wt = rand(m, k, 2, 2, seed=14) * 0.2
    assert_close(irdu.kernels.conv2x2s2(x.to(DEV), wt.to(DEV)), torch.nn.functional.conv2d(x, wt, stride=2), 1e-5)


@pytest.mark.parametrize("bchw", [(2, 3, 16, 20), (1, 3, 5, 7)])   # 16-byte path / scalar path
def test_repeat_graphs(irdu, bchw):
    b, c, h, w = bchw
    img = rand(b, c, h, w, seed=16)
    got = irdu.kernels.repeat_graphs(img.to(DEV), 5).cpu()
    assert torch.equal(got, img.repeat(1, 5, 1, 1))


def test_replicated_input_folding(irdu):
    """The image filter runs the 2x2/s2 conv and the pooled rhs on the un-replicated image
    (weights summed over the G replicas); the result must match the plain replicated path."""
    torch.manual_seed(3)
    g = 8
    mix = irdu.MixtureGTVGLR(g, 3, 0.5, 0.1, [[1e-3], [1e-4]], [[1e-4], [1e-4]], [[1e-4], [1e-4]],
                             n_cgd_iters=4, feature_extractor="v13")
    perturb_mixture(mix, 7)
    img = rand(2, 3, 24, 32, seed=17).to(DEV)
    mix = mix.to(DEV)
    with torch.no_grad():
        y = irdu.kernels.repeat_graphs(img, g)
        plain = mix(y)
        folded = mix(y, _src=img)
        unmaterialised = mix._solve(None, None, img)      # y never built: rhs A/B, skip read img
    assert_close(folded, plain, 1e-5)
    assert_close(unmaterialised, plain, 1e-5)


# The replicated first block (input = Cs channels copied R times) as one fused pass (lnb_rep_kernel:
# im2col GEMM1 with the depthwise folded in, gate + W2 in registers): against float64, with fp32-class
# error, for Cs = 1 / 2 / 3, a partial chunk (hid = 20), a tail workgroup (H * W not a multiple of 256),
# gray pixels (equal channels: sigma = sqrt(1e-5), the large-|x / sigma| exponent correction), and the
# skip from src (x = None) or from the materialised replicas.
@pytest.mark.parametrize("cs_r_hid_hw", [(3, 32, 256, (40, 36)), (3, 8, 20, (9, 13)), (1, 16, 48, (17, 30)),
                                         (2, 12, 64, (8, 8))])
@pytest.mark.parametrize("gray", [False, True])
def test_replicated_lnb_fused(irdu, cs_r_hid_hw, gray):
    cs, r, hid, (h, w) = cs_r_hid_hw
    c = cs * r
    assert irdu._native.load().grr_lnb_rep_fused(cs, r, c, hid) == 1
    torch.manual_seed(9)
    blk = irdu.LocalNonLinearBlock(c, hid, 1)
    with torch.no_grad():
        blk.skip_weight.copy_(torch.tensor([0.8, 1.2]))
        blk.norm.weighted_transform.weight.mul_(1.0 + 0.2 * torch.randn_like(blk.norm.weighted_transform.weight))
        blk.local_linear.channels_local_linear_op.weight.mul_(3.0)
    src = rand(2, cs, h, w, seed=19)
    if gray:
        src[:, :, : h // 2] = src[:, :1, : h // 2]          # upper half: equal channels
    x = src.repeat(1, r, 1, 1)
    p64 = {k: v.double() for k, v in sd_cpu(blk).items()}
    ref64 = O.local_nonlinear_block(x.double(), p64, "")
    err32 = rel_err(O.local_nonlinear_block(x, sd_cpu(blk), ""), ref64)
    blk = blk.to(DEV)
    with torch.no_grad():
        for xin in (None, x.to(DEV)):
            got = blk.forward_replicated(src.to(DEV), xin)
            err = rel_err(got, ref64)
            assert err <= 4 * err32 + 1e-6, (err, err32)


# (C, hid, H, W): C <= 128 runs the split-bf16 head (32 x 13 / 32 x 9 output tiles with halo
# recompute) + mix kernels: full / partial tiles, H*W % 4 == 0 (16-byte g DMA) and not (dword
# DMA), hid % 8 != 0 and hid % 16 != 0 (partial chunk / k-step), C = 33 (partial k-step and
# row tile), C = 128 (4 k-steps: 3 blocks per wave), tiny images (tile wider than the image);
# C = 160 / 192 run the fp32 MFMA path (v1.0 encoder/decoder widths).
@pytest.mark.parametrize("chw", [(12, 32, 16, 16), (96, 256, 40, 36), (33, 20, 9, 44), (24, 64, 13, 30),
                                 (128, 24, 8, 68), (6, 16, 5, 4), (96, 256, 27, 70), (64, 40, 1, 3),
                                 (160, 48, 12, 20), (192, 64, 9, 11), (384, 96, 6, 10)])
def test_local_nonlinear_block(irdu, chw):
    c, hid, h, w = chw
    torch.manual_seed(0)
    blk = irdu.LocalNonLinearBlock(c, hid, 1)
    with torch.no_grad():
        blk.skip_weight.copy_(torch.tensor([0.9, 1.3]))
        blk.norm.weighted_transform.weight.mul_(1.0 + 0.2 * torch.randn_like(blk.norm.weighted_transform.weight))
    x = rand(2, c, h, w, seed=15)
    ref = O.local_nonlinear_block(x, sd_cpu(blk), "")
    with torch.no_grad():
        got = blk.to(DEV)(x.to(DEV))
    assert_close(got, ref)


def _lnb_gate64(x64, p64):
    """The block's gated activation sigmoid(m) m v in float64 (the oracle's op sequence)."""
    n = O.custom_layer_norm(x64, p64, "norm.", 1)
    h = torch.nn.functional.conv2d(n, p64["local_linear.channels_linear_op.weight"])
    hp = torch.nn.functional.pad(h, (1, 1, 1, 1), mode="replicate")
    h = torch.nn.functional.conv2d(hp, p64["local_linear.channels_local_linear_op.weight"], groups=h.shape[1])
    m, v = h.chunk(2, dim=1)
    return torch.sigmoid(m) * m * v


# C <= 96: the whole block in one fused pass (lnb_fused16_kernel: GEMM1 / depthwise / gate / GEMM2 with the
# gated activation on chip).  Against float64 with fp32-class error: every k-step count (C = 6 ... 96),
# hid not a multiple of 16 (a partial last chunk), tiles past the image's right / bottom edge, one-row and
# one-column images, and a chunk-to-chunk magnitude ramp of the gated values (later chunks up to 2^12 x
# larger: the consumer's running exponent has to scale its accumulators down) plus gray pixels (equal
# channels: the large-|x / sigma| exponent correction of GEMM1's operand).
@pytest.mark.parametrize("c_hid_hw", [(96, 256, (40, 36)), (48, 96, (33, 70)), (6, 20, (5, 4)), (33, 40, (9, 44)),
                                      (96, 48, (1, 97)), (80, 64, (17, 1)), (64, 256, (8, 32)), (24, 64, (13, 30))])
@pytest.mark.parametrize("ramp", [False, True])
def test_fused_lnb_fp32_accurate(irdu, c_hid_hw, ramp):
    c, hid, (h, w) = c_hid_hw
    assert irdu._native.load().grr_lnb_fused(c, hid) == 1
    torch.manual_seed(11)
    blk = irdu.LocalNonLinearBlock(c, hid, 1)
    with torch.no_grad():
        blk.skip_weight.copy_(torch.tensor([0.7, 1.4]))
        blk.norm.weighted_transform.weight.mul_(1.0 + 0.2 * torch.randn_like(blk.norm.weighted_transform.weight))
        if ramp:
            w1 = blk.local_linear.channels_linear_op.weight
            scale = torch.pow(2.0, torch.arange(hid, dtype=torch.float32) // 16 * 1.5).clamp(max=4096.0)
            w1[:hid] *= scale.view(-1, 1, 1, 1)
            w1[hid:] *= scale.view(-1, 1, 1, 1)
    x = rand(2, c, h, w, seed=41, scale=2.0, offset=-0.3)
    if ramp:
        x[:, :, : max(1, h // 2)] = x[:, :1, : max(1, h // 2)]       # gray rows
    p64 = {k: v.double() for k, v in sd_cpu(blk).items()}
    ref64 = O.local_nonlinear_block(x.double(), p64, "")
    err32 = rel_err(O.local_nonlinear_block(x, sd_cpu(blk), ""), ref64)
    with torch.no_grad():
        got = blk.to(DEV)(x.to(DEV))
    err = rel_err(got, ref64)
    assert err <= 4 * err32 + 1e-6, (err, err32)
    # the training forward's kept gate (grr_lnb_forward_keep): the same pass also stores g
    ll = blk.local_linear
    with torch.no_grad():
        out_k, gate = irdu.kernels.lnb_forward_keep(
            x.to(DEV), blk.norm.weighted_transform.weight.view(c), ll.channels_linear_op.weight.view(2 * hid, c),
            ll.channels_local_linear_op.weight.view(2 * hid, 9), ll.project_out.weight.view(c, hid), blk.skip_weight)
    assert torch.equal(out_k, got)
    g64 = _lnb_gate64(x.double(), {k[len(""):]: v for k, v in p64.items()})
    assert rel_err(gate, g64) <= 1e-5, rel_err(gate, g64)


# ---------------------------------------------------------------------------
# full solver against the reference's golden vectors
@pytest.mark.parametrize("name", ["mixture_v1.npz", "mixture_v1_rect.npz"])
def test_mixture_golden(irdu, variant, name):
    d = load_golden(name)
    g = int(d["meta/n_graphs"])
    x = torch.from_numpy(d["in/x"])
    c = x.shape[1]
    m = irdu.MixtureGTVGLR(g, c // g, 0.5, 0.1, [[0.001], [0.0001]], [[0.0001], [0.0001]], [[0.0001], [0.0001]])
    m.load_state_dict(params_of(d, ""))
    with torch.no_grad():
        y = m.to(DEV)(x.to(DEV))
    assert_close(y, d["out/y"])


def test_msgf_v13_golden(irdu):
    d = load_golden("msgf_v13.npz")
    m = irdu.MultiScaleGraphFilter(3, 3, ngraphs=int(d["meta/n_graphs"]))
    m.load_state_dict(params_of(d, ""))
    with torch.no_grad():
        y = m.to(DEV)(torch.from_numpy(d["in/noisy"]).to(DEV))
    assert_close(y, d["out/y"])
    clean = torch.from_numpy(d["in/clean"])
    assert abs(O.psnr_ubyte(y.cpu(), clean) - O.psnr_ubyte(torch.from_numpy(d["out/y"]), clean)) <= 0.01


def test_abstract_model_golden(irdu):
    d = load_golden("abstract_v1.npz")
    cfg = {k[5:]: d[k] for k in d.files if k.startswith("meta/") and k != "meta/n_state_keys"}
    m = irdu.AbtractMultiScaleGraphFilter(
        n_channels_in=3, n_channels_out=3, dims=cfg["dims"].tolist(), hidden_dims=cfg["hidden_dims"].tolist(),
        nsubnets=cfg["nsubnets"].tolist(), ngraphs=cfg["ngraphs"].tolist(), num_blocks=cfg["num_blocks"].tolist(),
        num_blocks_out=int(cfg["num_blocks_out"]))
    m.load_state_dict(params_of(d, ""))
    m = m.to(DEV)
    img = torch.from_numpy(d["in/noisy"]).to(DEV)
    with torch.no_grad():
        coefs = m.encode(img)
        filt = m.filtering(coefs)
        y = m(img)
    for i in range(4):
        assert_close(filt[i], d[f"out/filtered{i}"])
    assert_close(y, d["out/y"])


# ---------------------------------------------------------------------------
# S = 10 stages (the metric's configuration) against the oracle
@pytest.mark.parametrize("case", [dict(g=4, b=2, h=32, w=32), dict(g=32, b=1, h=64, w=96),
                                  dict(g=4, b=1, h=24, w=256), dict(g=4, b=1, h=16, w=300),
                                  dict(g=4, b=1, h=20, w=512)])
def test_msgf_ten_stages_vs_oracle(irdu, variant, case):
    g, b, h, w = case["g"], case["b"], case["h"], case["w"]
    torch.manual_seed(2204)
    m = irdu.MultiScaleGraphFilter(3, 3, ngraphs=g, n_cgd_iters=10)
    perturb_mixture(m.localfilter, 21)
    clean = torch.rand(b, 3, h, w)
    noisy = clean + torch.randn(b, 3, h, w) * (25.0 / 255.0)
    ref = O.multiscale_graph_filter(noisy, sd_cpu(m), g)
    with torch.no_grad():
        got = m.to(DEV)(noisy.to(DEV))
    assert_close(got, ref)
    assert abs(O.psnr_ubyte(got.cpu(), clean) - O.psnr_ubyte(ref, clean)) <= 0.01


def test_c3_full_patch_sigma50_vs_oracle(irdu):
    """Config C3's per-patch workload at full size: one 256x256 RGB patch, sigma = 50, G = 32,
    S = 10 (the oracle finishes in seconds for one patch)."""
    torch.manual_seed(2250)
    m = irdu.MultiScaleGraphFilter(3, 3, ngraphs=32, n_cgd_iters=10)
    perturb_mixture(m.localfilter, 50)
    clean = torch.rand(1, 3, 256, 256)
    noisy = clean + torch.randn(1, 3, 256, 256) * (50.0 / 255.0)
    ref = O.multiscale_graph_filter(noisy, sd_cpu(m), 32)
    with torch.no_grad():
        got = m.to(DEV)(noisy.to(DEV))
    assert_close(got, ref)
    assert abs(O.psnr_ubyte(got.cpu(), clean) - O.psnr_ubyte(ref, clean)) <= 0.01


def test_full_batch_is_patch_independent(irdu):
    """Size-independent property at the bench's full shape (64 x 256x256, G = 32, S = 10): every
    patch of the batch filters exactly as it does alone, which is what batch sharding over GPUs
    relies on (no collective in the data path).  Bit-exact: no kernel mixes batch items."""
    torch.manual_seed(2251)
    m = irdu.MultiScaleGraphFilter(3, 3, ngraphs=32, n_cgd_iters=10)
    perturb_mixture(m.localfilter, 51)
    m = m.to(DEV)
    noisy = (torch.rand(64, 3, 256, 256) + torch.randn(64, 3, 256, 256) * (25.0 / 255.0)).to(DEV)
    with torch.no_grad():
        full = m(noisy)
        for i in (0, 17, 63):
            assert torch.equal(m(noisy[i:i + 1].contiguous())[0], full[i])
        assert torch.equal(m(noisy[32:40].contiguous()), full[32:40])
    assert torch.isfinite(full).all()


def test_lowpass_block_ten_stages_vs_oracle(irdu):
    torch.manual_seed(7)
    blk = irdu.LocalLowpassFilteringBlock(dim=48, nsubnets=1, ngraphs=8, n_cgd_iters=10)
    perturb_mixture(blk.local_filter, 31)
    with torch.no_grad():
        blk.skip_weight.copy_(torch.tensor([0.3, 0.8]))
    x = rand(2, 48, 48, 64, seed=17)
    ref = O.lowpass_block(x, sd_cpu(blk), 8)
    with torch.no_grad():
        got = blk.to(DEV)(x.to(DEV))
    assert_close(got, ref)


def test_single_stage_and_odd_half_level(irdu, variant):
    """S = 1 (the example.yaml plumbing config) and a half level with odd size (42x62 -> 21x31)."""
    torch.manual_seed(3)
    blk = irdu.LocalLowpassFilteringBlock(dim=12, nsubnets=1, ngraphs=4, n_cgd_iters=1)
    perturb_mixture(blk.local_filter, 41)
    x = rand(1, 12, 42, 62, seed=18)
    ref = O.lowpass_block(x, sd_cpu(blk), 4)
    with torch.no_grad():
        got = blk.to(DEV)(x.to(DEV))
    assert_close(got, ref)


def test_backward_fails_loudly(irdu):
    """The fused inference forward of LocalNonLinearBlock (``_forward_hip``, no saved state for a
    reverse; training goes through LNBFn instead) raises in backward if reached with autograd
    on, instead of silently dropping gradients."""
    blk = irdu.LocalNonLinearBlock(8, 16, 1).to(DEV)
    x = torch.rand(1, 8, 16, 16, device=DEV, requires_grad=True)
    y = blk._forward_hip(x)
    with pytest.raises(NotImplementedError):
        y.sum().backward()


# ---------------------------------------------------------------------------
# GLR-only v10 MixtureGLR (config C2 pattern)
@pytest.mark.parametrize("name", ["mixture_glr_v10.npz", "mixture_glr_v10_f1.npz"])
def test_mixture_glr_v10_golden(irdu, variant, name):
    d = load_golden(name)
    g = int(d["meta/n_graphs"])
    x = torch.from_numpy(d["in/x"])
    mix = irdu.MixtureGLR(g, x.shape[1] // g, 0.5, 0.1, [[0.001]])
    mix.load_state_dict(params_of(d, ""))
    with torch.no_grad():
        got = mix.to(DEV)(x.to(DEV))
    assert_close(got, d["out/y"])


@pytest.mark.parametrize("case", [dict(b=2, h=64, w=64), dict(b=1, h=40, w=300)])
def test_glr_image_filter_five_stages(irdu, variant, case):
    """Config C2 shape family: gray image, G = 8 graphs x F = 1, S = 5 stages, vs the oracle."""
    torch.manual_seed(12)
    m = irdu.GLRImageFilter(1, 1, ngraphs=8, n_cgd_iters=5)
    gen = torch.Generator().manual_seed(13)
    with torch.no_grad():
        lf = m.localfilter
        lf.alphaCGD.copy_(0.2 + 0.6 * torch.rand(lf.alphaCGD.shape, generator=gen))
        lf.betaCGD.copy_(0.05 + 0.35 * torch.rand(lf.betaCGD.shape, generator=gen))
        lf.muys00.copy_(0.05 + 0.55 * torch.rand(lf.muys00.shape, generator=gen))
    perturbed_graph_module(lf.GLRmodule00, 14)
    clean = torch.rand(case["b"], 1, case["h"], case["w"])
    noisy = clean + torch.randn(clean.shape) * (25.0 / 255.0)
    p = sd_cpu(m)
    x = noisy.repeat(1, 8, 1, 1)
    ref = torch.nn.functional.conv2d(O.mixture_glr_forward(x, O.sub_params(p, "localfilter."), 8),
                                     p["linear_combination.weight"])
    with torch.no_grad():
        got = m.to(DEV)(noisy.to(DEV))
    assert_close(got, ref)


# ---------------------------------------------------------------------------
# training parity against the reference's own autograd gradients (golden)
@pytest.mark.parametrize("name", ["mixture_v1.npz", "mixture_v1_rect.npz"])
def test_mixture_grad_vs_reference_golden(irdu, name):
    """L1-loss gradients of MixtureGTVGLR (input + every parameter) from the HIP reverse
    sweep vs the gradients the reference's PyTorch autograd produced (fixture)."""
    d = load_golden(name)
    g = int(d["meta/n_graphs"])
    x = torch.from_numpy(d["in/x"])
    mix = irdu.MixtureGTVGLR(g, x.shape[1] // g, 0.5, 0.1, [[1e-3], [1e-4]], [[1e-4], [1e-4]], [[1e-4], [1e-4]])
    mix.load_state_dict(params_of(d, ""))
    mix = mix.to(DEV)
    xg = x.to(DEV).requires_grad_(True)
    loss = torch.nn.functional.l1_loss(mix(xg), torch.from_numpy(d["in/target"]).to(DEV))
    loss.backward()
    assert abs(float(loss.detach()) - float(d["out/loss"])) <= 1e-5 * abs(float(d["out/loss"]))
    assert_close(xg.grad, d["grad/x"], 2e-4)
    for k, p in mix.named_parameters():
        assert_close(p.grad, d["grad/" + k], 2e-4)


@pytest.mark.parametrize("name", ["mixture_glr_v10.npz", "mixture_glr_v10_f1.npz"])
def test_mixture_glr_v10_grad_vs_reference_golden(irdu, name):
    """v10 MixtureGLR L1-loss gradients (HIP reverse) vs the reference's autograd gradients."""
    d = load_golden(name)
    g = int(d["meta/n_graphs"])
    x = torch.from_numpy(d["in/x"])
    mix = irdu.MixtureGLR(g, x.shape[1] // g, 0.5, 0.1, [[0.001]])
    mix.load_state_dict(params_of(d, ""))
    mix = mix.to(DEV)
    xg = x.to(DEV).requires_grad_(True)
    torch.nn.functional.l1_loss(mix(xg), torch.from_numpy(d["in/target"]).to(DEV)).backward()
    assert_close(xg.grad, d["grad/x"], 2e-4)
    # with F = 1 the normalised feature is sign(f) (REF:146-157): the feature-conv gradient is 0
    # analytically and both sides hold rounding noise (~1e-9), so errors are measured against
    # max(|ref|, 1e-4 x the largest parameter gradient)
    floor = 1e-4 * max(float(abs(d["grad/" + k]).max()) for k, _ in mix.named_parameters())
    for k, p in mix.named_parameters():
        ref = torch.from_numpy(d["grad/" + k]).double()
        err = float((p.grad.detach().double().cpu() - ref).abs().max()) / max(float(ref.abs().max()), floor)
        assert err <= 2e-4, (k, err)


def test_graph_module_sub_api_grads(irdu):
    """GLRFast / GTVFast forward and extract_edge_weights (the reference's sub-API) under
    autograd vs the fp64 oracle: gradients of input, edge weights and every parameter."""
    from tests.test_gpu_grad import weights_r
    torch.manual_seed(21)
    b, g, f, h, w = 2, 3, 4, 14, 18
    feat = rand(b, g, f, h, w, seed=22)
    x = rand(b, g, f, h, w, seed=23)
    for cls, apply in ((irdu.GLRFast, O.glr_apply), (irdu.GTVFast, O.gtv_apply)):
        m = perturbed_graph_module(cls(f, g, M_diag_init=1.0), 24)
        torch.set_default_dtype(torch.float64)
        try:
            p = {k: v.detach().double().requires_grad_(True) for k, v in m.state_dict().items()}
            fd, xd = feat.double().requires_grad_(True), x.double().requires_grad_(True)
            wgt, _ = O.edge_weights(fd, p["multiM"])
            out = apply(xd, wgt, O.stats_kernel(p, ""))
            (out * weights_r(out.shape).double()).sum().backward()
        finally:
            torch.set_default_dtype(torch.float32)
        m = m.to(DEV)
        fg, xg = feat.to(DEV).requires_grad_(True), x.to(DEV).requires_grad_(True)
        wg, _ = m.extract_edge_weights(fg)
        og = m(xg, wg)
        (og * weights_r(og.shape).to(DEV)).sum().backward()
        assert_close(og, out.detach(), 1e-5)
        assert_close(xg.grad, xd.grad, 2e-4)
        assert_close(fg.grad, fd.grad, 2e-4)
        for k, prm in m.named_parameters():
            assert_close(prm.grad, p[k].grad, 2e-4)


@pytest.mark.parametrize("bgfhw", [(64, 32, 3, 256, 256), (64, 32, 3, 128, 128), (16, 8, 3, 100, 128),
                                   (4, 8, 6, 96, 64), (2, 4, 1, 130, 200)])
def test_edge_weights_block_batch_independent_bitwise(irdu, bgfhw):
    """The edge-weight row kernel splits planes into row segments by a count that depends on the
    batch (>= 8192 waves), so a patch's weights come from different segment boundaries alone and
    in a batch; the prologue normalises a segment's first rows with the same explicit-fma
    arithmetic as the row loop, so the results must be bit-identical (H = 100 / 130: segments of
    unequal length; the single patch runs 8 segments, the full batch 1-2)."""
    b, g, f, h, w = bgfhw
    gen = torch.Generator().manual_seed(h + w)
    feat = torch.randn(b, 2 * g * f, h, w, generator=gen).to(DEV)
    mg, ml = ((torch.rand(g, f, generator=gen) + 0.5).to(DEV) for _ in range(2))
    full = irdu.kernels.edge_weights_block(feat, g, f, mg, ml)
    for i in (0, b - 1):
        one = irdu.kernels.edge_weights_block(feat[i:i + 1].contiguous(), g, f, mg, ml)
        for name, a, o in zip(("wG", "cG", "wL"), full, one):
            assert torch.equal(a[i], o[0]), (name, i)


# ---------------------------------------------------------------------------
# GLRFast / GTVFast sub-API methods (REF:128-228, :452-516) against the reference's own outputs
def test_sub_api_golden(irdu):
    d = load_golden("ops_small.npz")
    feat = torch.from_numpy(d["in/feat"]).to(DEV)
    x = torch.from_numpy(d["in/x"]).to(DEV)
    b, g, f, h, w = x.shape
    glr = irdu.GLRFast(f, g, 1.0)
    gtv = irdu.GTVFast(f, g, 1.0)
    glr.load_state_dict(params_of(d, "glr."))
    gtv.load_state_dict(params_of(d, "gtv."))
    glr, gtv = glr.to(DEV), gtv.to(DEV)
    with torch.no_grad():
        wl, dl = glr.extract_edge_weights(feat)
        wg, dg = gtv.extract_edge_weights(feat)
        assert_close(glr.stats_conv(x), d["out/glr_stats_conv"], 1e-5)
        assert_close(glr.stats_conv_transpose(x), d["out/glr_stats_conv_t"], 1e-5)
        assert_close(glr.op_L_norm(x, wl, dl), d["out/glr_op_L_norm"], 1e-5)
        e = gtv.op_C(x, wg, dg)
        assert_close(e, d["out/gtv_op_C"], 1e-5)
        # op_C_transpose on the reference's own edge signals and on ours
        assert_close(gtv.op_C_transpose(torch.from_numpy(d["out/gtv_op_C"]).to(DEV), wg, dg),
                     d["out/gtv_op_C_transpose"], 1e-5)
        assert_close(gtv.op_C_transpose(e, wg, dg), d["out/gtv_op_C_transpose"], 1e-5)
        # composition = forward (REF:518-523, :231-237)
        assert_close(gtv.op_C_transpose(gtv.op_C(x, wg), wg), gtv(x, wg), 1e-5)
        assert_close(glr.stats_conv_transpose(glr.op_L_norm(glr.stats_conv(x), wl)), glr(x, wl), 1e-5)
        # neighbour gather: the golden table is the gather of the flat index image
        idx = torch.arange(h * w, dtype=torch.float32, device=DEV).view(1, 1, h, w)
        nb = glr.get_neighbors_pixels(idx)
        assert np.array_equal(nb[0, 0].to(torch.int32).cpu().numpy(), d["out/neighbor_table"])
        # normalise + transform: the edge weights are its 4-way softmax of neighbour dot products
        fn = glr.normalize_and_transform_features(feat).cpu()
        assert_close(fn, O.normalize_features(feat.cpu(), glr.multiM.detach().cpu()), 1e-6)


@pytest.mark.parametrize("shape", [(2, 3, 4, 17, 23), (1, 2, 6, 40, 300), (1, 1, 1, 1, 5)])
def test_sub_api_random_vs_oracle(irdu, shape):
    """Odd sizes, one-row images and W > 256 against the oracle restatement of the same methods."""
    b, g, f, h, w = shape
    x = rand(b, g, f, h, w, seed=61)
    feat = rand(b, g, f, h, w, seed=62)
    wl = torch.softmax(rand(b, g, 4, h, w, seed=63), dim=2)
    glr = perturbed_graph_module(irdu.GLRFast(f, g, 1.0), 64)
    gtv = perturbed_graph_module(irdu.GTVFast(f, g, 1.0), 65)
    kl, kg = O.stats_kernel(sd_cpu(glr), ""), O.stats_kernel(sd_cpu(gtv), "")
    glr, gtv = glr.to(DEV), gtv.to(DEV)
    xd, wd = x.to(DEV), wl.to(DEV)
    with torch.no_grad():
        assert_close(glr.stats_conv(xd), O.stats_conv(x, kl), 1e-5)
        assert_close(glr.stats_conv_transpose(xd), O.stats_conv_t(x, kl), 1e-5)
        ref_l = x - torch.einsum("bgfehw,bgehw->bgfhw", O.gather_neighbors(x.reshape(b, g * f, h, w)).view(
            b, g, f, 4, h, w), wl)
        assert_close(glr.op_L_norm(xd, wd), ref_l, 1e-5)
        e = gtv.op_C(xd, wd)
        assert_close(e, O.gtv_C(x, wl, kg), 1e-5)
        assert_close(gtv.op_C_transpose(e, wd), O.gtv_Ct(e.cpu(), wl, kg), 1e-5)
        assert torch.equal(glr.get_neighbors_pixels(xd.reshape(b, g * f, h, w)).cpu(),
                           O.gather_neighbors(x.reshape(b, g * f, h, w)))
        assert_close(glr.normalize_and_transform_features(feat.to(DEV)),
                     O.normalize_features(feat, glr.multiM.detach().cpu()), 1e-6)
