"""PSNR parity on weights that denoise (the metric's "PSNR within 0.01 dB of reference").

No reference checkpoint exists, so scripts/train_psnr_fixture.py trained the bench's image filter
(MultiScaleGraphFilter G=32 F=3 S=10) on the HIP training path for 4,000 Adam steps on synthetic
sigma-25 patches; the weights are the committed fixture tests/golden/msgf_trained_g32_s10.safetensors
(loaded weights-only).  On held-out patches (a different generator and seed than the training
data) the HIP forward must match the CPU oracle within 1e-4 relative and 0.01 dB, while actually
denoising (output PSNR well above the noisy input's).

Soft-threshold branch flips (REF:684-704 is discontinuous at |C x| = gamma): the prox input
C x_1 is evaluated in float64 from the HIP stage-1 iterate and from the oracle's; the test prints
how many edge entries take a different branch of the threshold and bounds them.
"""
import os

import pytest
import torch

from oracle import graph_oracle as O
from tests.test_gpu_parity import DEV, rel_err

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURE = os.path.join(ROOT, "tests", "golden", "msgf_trained_g32_s10.safetensors")


@pytest.fixture(scope="module")
def trained():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import irdu_amd
    from bench import build_model
    irdu_amd.load_native()
    assert os.path.exists(FIXTURE), "weights fixture missing (scripts/train_psnr_fixture.py)"
    m = build_model(torch.device("cpu"), trained=True)
    state = {k: v.detach().clone() for k, v in m.state_dict().items()}
    return m.to(DEV).eval(), state


def test_trained_filter_psnr_parity(trained):
    from bench import synthetic_patches
    m, state = trained
    clean, noisy = synthetic_patches(2, seed=77)
    with torch.no_grad():
        got = m(noisy.to(DEV)).cpu()
    ref = O.multiscale_graph_filter(noisy, state, 32)
    err = rel_err(got, ref)
    p_noisy, p_got, p_ref = O.psnr_ubyte(noisy, clean), O.psnr_ubyte(got, clean), O.psnr_ubyte(ref, clean)
    print(f"\ntrained filter: PSNR noisy {p_noisy:.3f} dB -> HIP {p_got:.4f} / oracle {p_ref:.4f} dB, rel err {err:.2e}")
    assert err <= 1e-4
    assert abs(p_got - p_ref) <= 0.01
    assert p_got >= p_noisy + 5.0, "the fixture does not denoise"


def test_trained_filter_soft_threshold_branch_flips(trained):
    """Count prox branch flips between the HIP and the oracle stage-1 iterates (float64 C x)."""
    import irdu_amd
    from bench import synthetic_patches
    m, state = trained
    _, noisy = synthetic_patches(1, seed=78)
    g = 32
    # HIP x_1: the same filter with one unrolled stage returns the stage-0 iterate
    m1 = irdu_amd.MultiScaleGraphFilter(3, 3, ngraphs=g, n_cgd_iters=1)
    sd1 = {k: (v[:1] if k.endswith(("alphaCGD", "betaCGD")) else v) for k, v in state.items()}
    m1.load_state_dict(sd1)
    m1 = m1.to(DEV).eval()
    with torch.no_grad():
        x1_hip = m1.localfilter._solve(None, None, noisy.to(DEV)).cpu().double()
    p = O.sub_params(state, "localfilter.")
    y = noisy[:, None].repeat(1, g, 1, 1, 1).reshape(1, 3 * g, 256, 256)
    f0, f1 = O.features_v13(y, p)
    x1_ref = O.mixture_solve(y, p, f0, f1, g, n_stages=1).double()
    assert rel_err(x1_hip, x1_ref) <= 1e-4
    gr = O._Graphs(p, f0, f1, g, 3)
    flips, total = 0, 0
    for wG, k, gam, pool in ((gr.wG0, gr.kG0, gr.ga0, False), (gr.wG1, gr.kG1, gr.ga1, True)):
        outs = []
        for x1 in (x1_hip, x1_ref):
            x = O.pool2(x1) if pool else x1
            b, c, h, w = x.shape
            t = O.gtv_C(x.view(b, g, 3, h, w), wG.double(), k.double())
            outs.append(t.abs() > gam.double()[None, :, None, None, None, None])
        flips += int((outs[0] != outs[1]).sum())
        total += outs[0].numel()
    print(f"\nsoft-threshold branch flips HIP vs oracle: {flips} of {total} edge entries "
          f"({flips / total:.2e}); thresholded fraction {float(outs[1].double().mean()):.3f}")
    assert flips <= 1e-4 * total
