"""Pin the CPU oracle (oracle/graph_oracle.py) against golden vectors from the reference.

The fixtures were produced by running the reference implementation itself
(tests/golden/make_golden.py).  Float tolerance: 1e-5 relative to the tensor's
max-abs (oracle and reference run the same fp32 op sequence on the same CPU
torch; differences are last-bit only).  The neighbour table is bit-exact.
"""
import numpy as np
import pytest
import torch

from oracle import graph_oracle as O
from tests.golden_io import load_golden, params_of


def close(a, b, rtol=1e-5):
    a = torch.as_tensor(a, dtype=torch.float64)
    b = torch.as_tensor(b, dtype=torch.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    scale = max(float(b.abs().max()), 1e-30)
    err = float((a - b).abs().max()) / scale
    assert err <= rtol, f"rel err {err:.3e} > {rtol}"


@pytest.fixture(scope="module")
def ops():
    return load_golden("ops_small.npz")


def test_edge_delta_and_neighbor_table_bit_exact(ops):
    assert np.array_equal(O.edge_delta().numpy(), ops["out/edge_delta"])
    h, w = ops["out/neighbor_table"].shape[-2:]
    assert np.array_equal(O.neighbor_table(h, w).numpy(), ops["out/neighbor_table"])


def test_edge_weights(ops):
    feat = torch.from_numpy(ops["in/feat"])
    for m in ("glr", "gtv"):
        p = params_of(ops, m + ".")
        w, d = O.edge_weights(feat, p["multiM"])
        close(w, ops[f"out/{m}_w"])
        close(d, ops[f"out/{m}_deg"])


def test_stats_conv_and_transpose(ops):
    x = torch.from_numpy(ops["in/x"])
    k = O.stats_kernel(params_of(ops, "glr."), "")
    close(O.stats_conv(x, k), ops["out/glr_stats_conv"])
    close(O.stats_conv_t(x, k), ops["out/glr_stats_conv_t"])


def test_glr_and_gtv_operators(ops):
    x = torch.from_numpy(ops["in/x"])
    pl, pg = params_of(ops, "glr."), params_of(ops, "gtv.")
    wl = torch.from_numpy(ops["out/glr_w"])
    wg = torch.from_numpy(ops["out/gtv_w"])
    kl, kg = O.stats_kernel(pl, ""), O.stats_kernel(pg, "")
    close(O.glr_apply(x, wl, kl), ops["out/glr_forward"])
    e = O.gtv_C(x, wg, kg)
    close(e, ops["out/gtv_op_C"])
    close(O.gtv_Ct(e, wg, kg), ops["out/gtv_op_C_transpose"])
    close(O.gtv_apply(x, wg, kg), ops["out/gtv_forward"])


@pytest.mark.parametrize("name", ["mixture_v1.npz", "mixture_v1_rect.npz"])
def test_mixture_forward(name):
    d = load_golden(name)
    p = params_of(d, "")
    x = torch.from_numpy(d["in/x"])
    g = int(d["meta/n_graphs"])
    close(O.mixture_forward(x, p, g, "v1"), d["out/y"], rtol=2e-5)


@pytest.mark.parametrize("name", ["mixture_v1.npz", "mixture_v1_rect.npz"])
def test_system_operator(name):
    d = load_golden(name)
    p = params_of(d, "")
    x = torch.from_numpy(d["in/x"])
    g = int(d["meta/n_graphs"])
    b, c, h, w = x.shape
    f0, f1 = O.features_v1(x, p)
    gr = O._Graphs(p, f0, f1, g, c // g)
    ax = O.system_operator(x.reshape(b, g, c // g, h, w), gr).reshape(b, c, h, w)
    close(ax, d["out/Ax"])


def test_mixture_gradients():
    d = load_golden("mixture_v1.npz")
    p = {k: v.clone().requires_grad_(True) for k, v in params_of(d, "").items()}
    x = torch.from_numpy(d["in/x"]).clone().requires_grad_(True)
    g = int(d["meta/n_graphs"])
    loss = torch.nn.functional.l1_loss(O.mixture_forward(x, p, g, "v1"), torch.from_numpy(d["in/target"]))
    loss.backward()
    assert abs(float(loss.detach()) - float(d["out/loss"])) <= 1e-6 * abs(float(d["out/loss"]))
    close(x.grad, d["grad/x"], rtol=1e-4)
    for k, v in p.items():
        key = "grad/" + k
        if key in d:
            close(v.grad, d[key], rtol=1e-4)


def test_multiscale_graph_filter_v13():
    d = load_golden("msgf_v13.npz")
    p = params_of(d, "")
    y = O.multiscale_graph_filter(torch.from_numpy(d["in/noisy"]), p, int(d["meta/n_graphs"]))
    close(y, d["out/y"], rtol=2e-5)


def test_abstract_model_v1():
    d = load_golden("abstract_v1.npz")
    p = params_of(d, "")
    img = torch.from_numpy(d["in/noisy"])
    nb = [int(v) for v in d["meta/num_blocks"]]
    ng = [int(v) for v in d["meta/ngraphs"]]
    coefs = O.abstract_encode(img, p, nb, (1, 1, 1, 1))
    for i in range(4):
        close(coefs[i], d[f"out/coef{i}"])
    filt = O.abstract_filtering(coefs, p, ng)
    for i in range(4):
        close(filt[i], d[f"out/filtered{i}"], rtol=2e-5)
    y = O.abstract_forward(img, p, ng, nb, int(d["meta/num_blocks_out"]))
    close(y, d["out/y"], rtol=2e-5)
    assert len([k for k in d.files if k.startswith("p/")]) == int(d["meta/n_state_keys"])


def test_psnr_helper():
    clean = torch.full((1, 3, 8, 8), 100.0 / 255.0)
    assert O.psnr_ubyte(clean, clean) == float("inf")
    noisy = clean + 2.2 / 255.0  # quantises to exactly +2 grey levels
    assert abs(O.psnr_ubyte(noisy, clean) - 20 * np.log10(255 / 2.0)) < 1e-9


@pytest.mark.parametrize("name", ["mixture_glr_v10.npz", "mixture_glr_v10_f1.npz"])
def test_mixture_glr_v10_forward_and_grads(name):
    """GLR-only v10 MixtureGLR (lib/model_GLR_GTV_deep_v10.py:241-335): forward and the
    reference's own L1-loss autograd gradients."""
    d = load_golden(name)
    g = int(d["meta/n_graphs"])
    p = {k: v.clone().requires_grad_(True) for k, v in params_of(d, "").items()}
    x = torch.from_numpy(d["in/x"]).requires_grad_(True)
    y = O.mixture_glr_forward(x, p, g)
    close(y.detach(), d["out/y"])
    torch.nn.functional.l1_loss(y, torch.from_numpy(d["in/target"])).backward()
    close(x.grad, d["grad/x"], 1e-4)
    for k, v in p.items():
        close(v.grad, d["grad/" + k], 1e-4)
