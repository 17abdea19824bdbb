"""grr_bwd_padj2: the x-gradient passes of a level's GLR and GTV terms in one sweep must equal the
two accumulating grr_bwd_stencil (mode P*) launches (same expressions and order; the compiler contracts
the scale-and-add differently in the two kernels, so to 2 ulp-scale: 1e-6 of the largest value), and
the training reverse with it must equal the reverse without it."""
import pytest
import torch

from tests.test_gpu_parity import DEV, perturb_mixture, rand

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def irdu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import irdu_amd
    irdu_amd.load_native()
    return irdu_amd


@pytest.mark.parametrize("bgfhw", [(2, 4, 3, 16, 32), (1, 2, 6, 9, 12), (2, 8, 3, 64, 256)])
def test_padj2_equals_two_stencil_passes(irdu, bgfhw):
    from irdu_amd import kernels as K
    b, g, f, h, w = bgfhw
    c = g * f
    v1, v2, out0 = (rand(b, c, h, w, seed=s).to(DEV) for s in (1, 2, 3))
    t1, t2 = rand(c, 5, seed=4).to(DEV), rand(c, 5, seed=5).to(DEV)
    s1, s2 = rand(g, seed=6).to(DEV), rand(g, seed=7).to(DEV)
    ref = out0.clone()
    K.bwd_stencil(v1, t1, K.ST_P_ADJ, g, s1, out=ref)
    K.bwd_stencil(v2, t2, K.ST_P_ADJ, g, s2, out=ref)
    got = out0.clone()
    K.bwd_padj2(v1, t1, s1, v2, t2, s2, got, g)
    err = float((got - ref).abs().max() / ref.abs().max())
    assert err <= 1e-6, err


def test_reverse_with_padj2_equals_without(irdu):
    import torch.nn.functional as F
    from irdu_amd import solver_grad as SG
    torch.manual_seed(4)
    blk = irdu.LocalLowpassFilteringBlock(dim=12, nsubnets=1, ngraphs=4, n_cgd_iters=4)
    perturb_mixture(blk.local_filter, 5)
    blk = blk.to(DEV)
    x, t = rand(2, 12, 32, 48, seed=8).to(DEV), rand(2, 12, 32, 48, seed=9).to(DEV)
    grads = []
    saved = SG.PADJ2
    try:
        for on in (False, True):
            SG.PADJ2 = on
            xa = x.clone().requires_grad_(True)
            for p in blk.parameters():
                p.grad = None
            F.l1_loss(blk(xa), t).backward()
            grads.append([xa.grad] + [p.grad.clone() for p in blk.parameters()])
    finally:
        SG.PADJ2 = saved
    for a, b in zip(*grads):
        # padj2_kernel evaluates the two accumulating stencil launches' expressions in their order and
        # the reductions are fixed-order (no float atomics): the tight round-2 floor holds again
        assert float((a - b).abs().max()) <= 1e-6 * float(b.abs().max()) + 1e-12
