"""Tiled (overlap-save) inference vs whole-image inference on the GPU (config C5 path)."""
import pytest
import torch

from tests.test_gpu_parity import DEV, perturb_mixture, rel_err

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def irdu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import irdu_amd
    irdu_amd.load_native()
    return irdu_amd


def test_tiled_equals_whole_image_when_halo_covers_receptive_field(irdu):
    """S = 1 block: receptive field < 32 px, so 32-px halos reproduce the whole-image result."""
    from irdu_amd import tiling
    torch.manual_seed(4)
    blk = irdu.LocalLowpassFilteringBlock(dim=12, nsubnets=1, ngraphs=4, n_cgd_iters=1)
    perturb_mixture(blk.local_filter, 44)
    blk = blk.to(DEV)
    x = torch.rand(1, 12, 192, 256, device=DEV)
    with torch.no_grad():
        whole = blk(x)
    tiled = tiling.tiled_forward(blk, x, tile=128, halo=32, align=16, micro_batch=4)
    assert rel_err(tiled, whole) <= 1e-5


def test_tiled_msgf_ten_stages_halo(irdu):
    """S = 10 image filter: its analytic receptive field is 83 px, but the
    solver's influence decays geometrically with distance, so 32- and 64-px halos already
    reproduce the whole image to fp32 rounding (the kernels differ between the window width and
    the image width, hence not bit-exact)."""
    from irdu_amd import tiling
    torch.manual_seed(5)
    m = irdu.MultiScaleGraphFilter(3, 3, ngraphs=8, n_cgd_iters=10)
    perturb_mixture(m.localfilter, 55)
    m = m.to(DEV)
    x = torch.rand(1, 3, 384, 384, device=DEV)
    with torch.no_grad():
        whole = m(x)
    errs = [rel_err(tiling.tiled_forward(m, x, tile=128 + 2 * hl, halo=hl, align=16), whole) for hl in (32, 64)]
    print("tiled vs whole rel err by halo 32/64:", errs)
    assert max(errs) <= 1e-5
