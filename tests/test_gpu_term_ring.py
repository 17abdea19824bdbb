"""grr_bwd_term_fused's LDS-ring row kernel (the operand rows of every step DMA'd into LDS by a producer
wave, grr_bwd_set_term_rows(2), the default) against the register-prefetch row kernel (level 1), for the
three operator terms: v and the weight gradient to 2e-6 (same expressions and order; the two
instances are compiled apart, so an FMA contraction may differ by an ulp), the per-graph / per-channel
reductions to fp32 summation-order accuracy (the ring kernel's column strips are 16-byte aligned:
64 V - 8 owned columns against 62 V).  Covers ring depths 4-6, one and two
workgroups per CU, segmented grids with ragged ends, one- to three-row images, F up to the ring's
limit (7 at 4-column lanes, 12 below) and shapes the ring does not take (W % 4 != 0, F above it),
which must fall back to the same result.  The register kernel is pinned against the per-pixel kernel
by test_gpu_term_rows.py."""
import pytest
import torch

from tests.test_gpu_parity import DEV, rel_err

pytestmark = pytest.mark.gpu

# (b, G, F, H, W): 4-column lanes (W 129..256 and strips), 2-column (65..128, strips for the GLR / prox
# terms at W > 256), 1-column (<= 64)
CASES = [(2, 4, 3, 20, 256), (1, 3, 1, 9, 32), (1, 2, 2, 17, 100), (1, 2, 4, 70, 200), (3, 2, 3, 2, 64),
         (1, 1, 3, 300, 128), (1, 2, 3, 11, 300), (1, 2, 4, 8, 512), (1, 1, 2, 6, 744), (2, 2, 6, 18, 256),
         (1, 2, 7, 9, 256), (1, 2, 12, 9, 128), (2, 1, 12, 12, 64), (1, 1, 6, 5, 32), (1, 2, 6, 7, 512),
         (1, 1, 12, 5, 300), (2, 3, 3, 1, 96), (1, 2, 5, 3, 248), (4, 8, 3, 64, 256),
         # not taken by the ring kernel: W % 4 != 0, F = 8 at 4-column lanes
         (1, 2, 3, 10, 102), (1, 2, 8, 6, 256)]


@pytest.fixture(scope="module")
def K():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import irdu_amd
    irdu_amd.load_native()
    from irdu_amd import kernels
    yield kernels
    kernels.set_term_rows(True)


def _run(K, level, mode, x, g, taps, w, lg, scale, G):
    K.set_term_rows(level)
    gw = torch.full_like(w, 0.5)           # accumulated into (+=)
    gdot = torch.full((G,), 0.25, device=DEV)
    ggam = torch.full((G,), -0.5, device=DEV) if mode == 2 else None
    gtaps = torch.zeros_like(taps)
    v = K.bwd_term_fused(mode, x, g, taps, w, lg, scale, 0.7, gw, ggam, gdot, gtaps, G)
    torch.cuda.synchronize()
    return v.cpu(), gw.cpu(), gdot.cpu(), None if ggam is None else ggam.cpu(), gtaps.cpu()


@pytest.mark.parametrize("case", CASES, ids=lambda c: "b{}g{}f{}h{}w{}".format(*c))
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_term_ring_equals_register_kernel(K, case, mode):
    b, G, F, h, w_ = case
    torch.manual_seed(mode * 1000 + 7 * h + w_ + F)
    C = G * F
    x = torch.randn(b, C, h, w_, device=DEV)
    g = torch.randn(b, C, h, w_, device=DEV)
    taps = torch.randn(C, 5, device=DEV) * 0.5
    w = torch.rand(b, G, 2 if mode == 1 else 4, h, w_, device=DEV)
    # a spread of |t| around gamma so the prox term's three branches all occur
    lg = torch.log(torch.linspace(0.05, 0.5, G, device=DEV)) if mode == 2 else None
    scale = torch.rand(G, device=DEV) + 0.5
    ref = _run(K, 1, mode, x, g, taps, w, lg, scale, G)
    got = _run(K, 2, mode, x, g, taps, w, lg, scale, G)
    for name, a, r in zip(["v", "gw", "gdot", "ggamma", "gtaps"], got, ref):
        if r is None:
            continue
        assert torch.isfinite(a).all(), name
        if name in ("v", "gw"):
            # same expressions, compiled per instance: the compiler's FMA contraction may differ by an ulp
            assert rel_err(a, r) <= 2e-6, (name, rel_err(a, r))
        else:
            n = b * F * h * w_
            sc = max(float(r.abs().max()), n ** 0.5)
            err = float((a.double() - r.double()).abs().max())
            assert err <= 2e-5 * sc, (name, err, sc)


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_term_ring_bitwise_reproducible(K, mode):
    """The ring kernel's outputs, reductions included, are identical run to run."""
    torch.manual_seed(40 + mode)
    b, G, F, h, w_ = 2, 4, 6, 37, 512
    C = G * F
    x = torch.randn(b, C, h, w_, device=DEV)
    g = torch.randn(b, C, h, w_, device=DEV)
    taps = torch.randn(C, 5, device=DEV) * 0.5
    w = torch.rand(b, G, 2 if mode == 1 else 4, h, w_, device=DEV)
    lg = torch.log(torch.linspace(0.05, 0.5, G, device=DEV)) if mode == 2 else None
    scale = torch.rand(G, device=DEV) + 0.5
    a = _run(K, 2, mode, x, g, taps, w, lg, scale, G)
    bb = _run(K, 2, mode, x, g, taps, w, lg, scale, G)
    for ta, tb in zip(a, bb):
        if ta is not None:
            assert torch.equal(ta, tb)


# W > 64 V whose last column strip owns <= 56 columns: the ring kernel runs that strip as a second,
# one-column-lane launch (grr_bwd_set_term_tail(1), the default).  (b, G, F, H, W): W = 512 (4-column lanes:
# 2 strips + a 16-column tail for the pair term; 2-column lanes: 4 + a 32-column tail for GLR / prox), W = 300
# (pair term: 248 + a 52-column tail), W = 744 (2-column lanes: 6 strips + 24), W = 400 (no tail: 152 / 40 owned)
TAIL_CASES = [(1, 2, 6, 7, 512), (2, 1, 3, 33, 512), (1, 2, 4, 8, 300), (1, 1, 2, 6, 744), (1, 2, 3, 5, 400)]


@pytest.mark.parametrize("case", TAIL_CASES, ids=lambda c: "b{}g{}f{}h{}w{}".format(*c))
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_term_ring_tail_equals_full_strips(K, case, mode):
    b, G, F, h, w_ = case
    torch.manual_seed(5000 + mode * 100 + h + w_)
    C = G * F
    x = torch.randn(b, C, h, w_, device=DEV)
    g = torch.randn(b, C, h, w_, device=DEV)
    taps = torch.randn(C, 5, device=DEV) * 0.5
    w = torch.rand(b, G, 2 if mode == 1 else 4, h, w_, device=DEV)
    lg = torch.log(torch.linspace(0.05, 0.5, G, device=DEV)) if mode == 2 else None
    scale = torch.rand(G, device=DEV) + 0.5
    try:
        K.set_term_tail(False)
        ref = _run(K, 2, mode, x, g, taps, w, lg, scale, G)
        K.set_term_tail(True)
        got = _run(K, 2, mode, x, g, taps, w, lg, scale, G)
        again = _run(K, 2, mode, x, g, taps, w, lg, scale, G)
    finally:
        K.set_term_tail(True)
    for name, a, r, a2 in zip(["v", "gw", "gdot", "ggamma", "gtaps"], got, ref, again):
        if r is None:
            continue
        assert torch.equal(a, a2), name           # fixed-order reductions across the two launches
        assert torch.isfinite(a).all(), name
        if name in ("v", "gw"):
            assert rel_err(a, r) <= 2e-6, (name, rel_err(a, r))
        else:
            n = b * F * h * w_
            sc = max(float(r.abs().max()), n ** 0.5)
            err = float((a.double() - r.double()).abs().max())
            assert err <= 2e-5 * sc, (name, err, sc)
