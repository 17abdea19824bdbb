"""Window-graph oracle (oracle/window_oracle.py) against the reference's own outputs.

Fixtures: tests/golden/window_ops_v7.npz, window_v7.npz, made by importing
REF7 = lib/model_GLR_GTV_deep_v7.py (tests/golden/make_golden_window.py).  CPU only.
"""
import numpy as np
import pytest
import torch

from oracle import window_oracle as O
from tests.golden_io import load_golden

WINDOWS = ("ring3", "diamond5", "full5")


def _rel(a, b):
    b = torch.as_tensor(np.asarray(b)).double()
    return float((a.double() - b).abs().max() / b.abs().max())


def _ops_params(d, name, pre):
    full = f"{name}/p/{pre}"
    return {k[len(full):]: torch.from_numpy(d[k].copy()) for k in d.files if k.startswith(full)}


@pytest.mark.parametrize("name", WINDOWS)
def test_window_edges_and_operators(name):
    d = load_golden("window_ops_v7.npz")
    delta = d[f"{name}/delta"]
    assert np.array_equal(O.window_edges({"ring3": np.array([1, 1, 1, 1, 0, 1, 1, 1, 1]).reshape(3, 3),
                                          "diamond5": np.array([0, 0, 1, 0, 0, 0, 1, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1,
                                                                1, 1, 0, 0, 0, 1, 0, 0]).reshape(5, 5),
                                          "full5": np.array([1] * 12 + [0] + [1] * 12).reshape(5, 5)}[name]), delta)
    pL, pG = _ops_params(d, name, "glr."), _ops_params(d, name, "gtv.")
    feat, x = torch.from_numpy(d[f"{name}/feat"]), torch.from_numpy(d[f"{name}/x"])
    wl, deg = O.edge_weights(feat, pL["multiM"], delta)
    wg, _ = O.edge_weights(feat, pG["multiM"], delta)
    assert _rel(wl, d[f"{name}/wL"]) <= 1e-6 and _rel(wg, d[f"{name}/wG"]) <= 1e-6
    assert _rel(deg, d[f"{name}/degL"]) <= 1e-6
    kL, kG = O.stats_kernel(pL, "", 3), O.stats_kernel(pG, "", 3)
    assert _rel(O.glr_apply(x, wl, kL, delta), d[f"{name}/glr"]) <= 1e-6
    assert _rel(O.gtv_C(x, wg, kG, delta), d[f"{name}/gtv_C"]) <= 1e-6
    assert _rel(O.gtv_Ct(O.gtv_C(x, wg, kG, delta), wg, kG, delta), d[f"{name}/gtv"]) <= 1e-6


def test_window_mixture_forward():
    g = load_golden("window_v7.npz")
    p = {k[2:]: torch.from_numpy(g[k].copy()) for k in g.files if k.startswith("p/")}
    out = O.mixture_gtv_v7(torch.from_numpy(g["in/noisy"]), p, 4, 3,
                           np.array([0, 0, 1, 0, 0, 0, 1, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 1, 0, 0, 0, 1, 0, 0])
                           .reshape(5, 5))
    assert _rel(out, g["out/y"]) <= 1e-5


def test_window_state_dict_keys_match_reference():
    import irdu_amd
    from irdu_amd import window_graph as WG
    g = load_golden("window_v7.npz")
    m = WG.MixtureGTV(3, 4, 3, 8, WG.CONNECTION_FLAGS_5x5_small, 4, 0.5, 0.1, torch.tensor([[0.1]]),
                      torch.tensor([[0.1]]), torch.tensor([[0.001]]))
    ref_keys = {k[2:] for k in g.files if k.startswith("p/")}
    assert set(m.state_dict().keys()) == ref_keys and len(ref_keys) == int(g["meta/n_state_keys"])
    m.load_state_dict({k: torch.from_numpy(g["p/" + k].copy()) for k in ref_keys}, strict=True)
    assert np.array_equal(WG.window_edges(WG.CONNECTION_FLAGS_5x5_small),
                          load_golden("window_ops_v7.npz")["diamond5/delta"])


def test_window_module_rejects_cpu_tensors():
    from irdu_amd import window_graph as WG
    glr = WG.GLRFast(3, 3, 2, WG.CONNECTION_FLAGS_3x3)
    with pytest.raises((RuntimeError, Exception)):
        with torch.no_grad():
            glr(torch.zeros(1, 2, 3, 8, 8), torch.zeros(1, 2, 8, 8, 8))


V1_WINDOWS = {"ring3": (2, 3, np.array([1, 1, 1, 1, 0, 1, 1, 1, 1]).reshape(3, 3)),
              "full5": (2, 2, np.array([1] * 12 + [0] + [1] * 12).reshape(5, 5))}


def _v1_params(d, pre):
    return {k[len(pre):]: torch.from_numpy(d[k].copy()) for k in d.files if k.startswith(pre)}


@pytest.mark.parametrize("name", sorted(V1_WINDOWS))
def test_window_v1_block_forward(name):
    """REF1 MixtureGTV (no stats stencils, 4-level feature U-Net, 6 CG stages) vs the reference."""
    d = load_golden("window_v1.npz")
    g, f, cw = V1_WINDOWS[name]
    out = O.mixture_gtv_v1(torch.from_numpy(d[f"{name}/in"]), _v1_params(d, f"{name}/p/"), g, f, cw)
    assert _rel(out, d[f"{name}/out"]) <= 1e-5


def test_window_v1_sharpening():
    d = load_golden("window_v1.npz")
    out = O.sharpening(torch.from_numpy(d["sharp/in"]), _v1_params(d, "sharp/p/"), "")
    assert _rel(out, d["sharp/out"]) <= 1e-6


def test_window_v1_state_dict_keys_match_reference():
    from irdu_amd import window_graph_v1 as W1
    d = load_golden("window_v1.npz")
    for name, (g, f, cw) in V1_WINDOWS.items():
        m = W1.MixtureGTV(3, g, f, cw, 6, 0.5, 0.1, torch.tensor([[0.1]]), torch.tensor([[0.1]]),
                          torch.tensor([[0.001]]))
        ref = _v1_params(d, f"{name}/p/")
        assert set(m.state_dict()) == set(ref) and len(ref) == int(d[f"{name}/meta/n_state_keys"])
        m.load_state_dict(ref, strict=True)
    W1.SharpeningBlock(3, 3, 24).load_state_dict(_v1_params(d, "sharp/p/"), strict=True)
    seq = W1.MultiScaleSequenceDenoiser()
    assert sum(1 for k in seq.state_dict() if k.endswith("alphaCGD")) == 3


def test_window_host_checks_reject_bad_shapes_without_gpu():
    """Shape errors surface on the host before any launch (CPU tensors would also be refused)."""
    from irdu_amd import kernels as K
    from irdu_amd import window_graph as WG
    delta = WG.window_edges(WG.CONNECTION_FLAGS_3x3)
    assert delta.shape == (8, 2)
    with pytest.raises(ValueError):
        K._check_win_scalars(4, ro=torch.zeros(3))
    with pytest.raises(ValueError):
        K._check_win_scalars(4, tapsG=torch.zeros(4))
    K._check_win_scalars(4, ro=torch.zeros(4), tapsG=torch.zeros(5), beta=None)
