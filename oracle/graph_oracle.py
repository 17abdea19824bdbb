"""CPU oracle for the GGTV/GGLR unrolled graph-filter hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / the timed CPU baseline.  The product path (``irdu_amd``) never calls
it and fails loudly when its HIP library is missing.

What it is: a from-scratch, functional (no nn.Module) restatement in PyTorch-CPU
fp32 of the reference algorithm in
``exploration/GGTV_GGLR_v1.0/deep_multiscale_GGLR_GGTV_v1x0.py`` (REF below; the
same file is byte-identical to ``lib/model_GLR_GTV_deep_v13.py``/``_v22.py``) and of
the image-domain feature CNN of ``lib/model_GLR_GTV_deep_v13_no_latent.py``
(REF13 below).  It follows the reference's op sequence (replicate pad, stacked
neighbour views, einsum-style scaling, softmax, ``where``) so that it is also a
fair CPU baseline of the reference's PyTorch-CPU path.

Parameters are passed as a flat ``dict`` keyed exactly like the reference's
``state_dict`` (e.g. ``"GLRmodule00.multiM"``), so a reference checkpoint's
``state_dict`` drives the oracle unchanged.  The constant 3x3 basis kernels and
the 2x2 scaling kernel, which the reference keeps as plain (non-state) tensors
(REF:56-118, :613), are rebuilt here.

Pinning: golden vectors produced by importing the reference itself in the build
container (``tests/golden/make_golden.py``) are checked against this module in
``tests/test_oracle_golden.py``.  Stage counts S > 3 have no literal reference
instance; they follow the reference's own extension pattern (REF:797-807) and
are pinned only through the S = 3 code path they share.
"""
from __future__ import annotations

import math
from typing import Callable, Dict, Optional, Sequence, Tuple

import torch
import torch.nn.functional as Fn

Tensor = torch.Tensor
Params = Dict[str, Tensor]

# ---------------------------------------------------------------------------
# a1: fixed 4-neighbour stencil.  REF:26-53 builds the 3x3 "small" connection
# window, enumerates offsets with itertools.product(m, m) (row-major over
# (dy, dx) in {-1,0,1}^2) and keeps the four flagged ones, in that order.
# ---------------------------------------------------------------------------
EDGE_DELTA = ((-1, 0), (0, -1), (0, 1), (1, 0))  # up, left, right, down
PAD_HW = (1, 1)  # REF:50  |min(edge_delta)| per axis


def edge_delta() -> Tensor:
    """int32 [4, 2] offsets (dy, dx) in the reference's edge order (REF:42-53)."""
    return torch.tensor(EDGE_DELTA, dtype=torch.int32)


def neighbor_table(h: int, w: int) -> Tensor:
    """int32 [4, h, w]: flat index (row*w + col) of the neighbour each edge reads.

    The reference reads neighbours from a replicate-padded frame (REF:128-144), i.e.
    neighbour e of pixel p is ``clamp(p + delta_e)`` into the image.
    """
    rows = torch.arange(h, dtype=torch.int64)[:, None].expand(h, w)
    cols = torch.arange(w, dtype=torch.int64)[None, :].expand(h, w)
    out = []
    for dy, dx in EDGE_DELTA:
        r = (rows + dy).clamp(0, h - 1)
        c = (cols + dx).clamp(0, w - 1)
        out.append(r * w + c)
    return torch.stack(out).to(torch.int32)


# ---------------------------------------------------------------------------
# a1/a5/a6: learned per-channel 3x3 "stats" stencil S (REF:56-118, :177-215)
# ---------------------------------------------------------------------------
def _basis_kernels() -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    z = torch.zeros(3, 3)
    k01 = z.clone(); k01[1, 1] = 1.0                       # REF:56-60 identity tap
    k02a = z.clone(); k02a[1, 1] = -1.0; k02a[1, 2] = 1.0  # REF:72-76 horizontal diff
    k02b = z.clone(); k02b[1, 1] = -1.0; k02b[2, 1] = 1.0  # REF:88-92 vertical diff
    k03 = torch.tensor([[0.0, -1.0, 0.0], [-1.0, 4.0, -1.0], [0.0, -1.0, 0.0]])  # REF:104-108
    return k01, k02a, k02b, k03


def stats_kernel(p: Params, prefix: str) -> Tensor:
    """[C,1,3,3] depthwise kernel = p01*k01 + p02a*k02a + p02b*k02b + p03*k03 (REF:178-183)."""
    k01, k02a, k02b, k03 = _basis_kernels()
    return (p[prefix + "stats_kernel_p01"] * k01
            + p[prefix + "stats_kernel_p02a"] * k02a
            + p[prefix + "stats_kernel_p02b"] * k02b
            + p[prefix + "stats_kernel_p03"] * k03)


def stats_conv(x5: Tensor, k: Tensor) -> Tensor:
    """S x: replicate pad 1 then depthwise 3x3 cross-correlation (REF:177-195)."""
    b, g, f, h, w = x5.shape
    xp = Fn.pad(x5.reshape(b, g * f, h, w), (1, 1, 1, 1), mode="replicate")
    return Fn.conv2d(xp, k, groups=g * f).view(b, g, f, h, w)


def stats_conv_t(x5: Tensor, k: Tensor) -> Tensor:
    """S^T x: conv_transpose2d(padding=1) of the same kernel, zero boundary (REF:197-215)."""
    b, g, f, h, w = x5.shape
    y = Fn.conv_transpose2d(x5.reshape(b, g * f, h, w), k, padding=1, groups=g * f)
    return y.view(b, g, f, h, w)


# ---------------------------------------------------------------------------
# a2-a4: neighbour gather and edge weights
# ---------------------------------------------------------------------------
def gather_neighbors(x4: Tensor) -> Tensor:
    """[B,C,H,W] -> [B,C,4,H,W], neighbour e = x(clamp(p+delta_e)) (REF:128-144)."""
    _, _, h, w = x4.shape
    ph, pw = PAD_HW
    frame = Fn.pad(x4, (pw, pw, ph, ph), mode="replicate")
    views = [frame[:, :, ph + dy:ph + dy + h, pw + dx:pw + dx + w] for dy, dx in EDGE_DELTA]
    return torch.stack(views, dim=-3)


def normalize_features(f5: Tensor, multiM: Tensor) -> Tensor:
    """L2-normalise over node features (eps 1e-12) then scale by multiM[g,f] (REF:146-157)."""
    b, g, f, h, w = f5.shape
    fn = Fn.normalize(f5, dim=2)
    return (fn * multiM[None, :, :, None, None]).reshape(b, g * f, h, w)


def edge_weights(f5: Tensor, multiM: Tensor) -> Tuple[Tensor, Tensor]:
    """Softmax-over-edges feature similarity (REF:160-175).

    Returns ``(w [B,G,4,H,W], degree [B,G,H,W])``; degree is the edge-sum of w.
    """
    b, g, f, h, w = f5.shape
    fh = normalize_features(f5, multiM)
    nb = gather_neighbors(fh)
    sim = (fh[:, :, None] * nb).view(b, g, f, 4, h, w).sum(dim=2)
    wgt = torch.softmax(sim, dim=2)
    return wgt, wgt.sum(dim=2)


# ---------------------------------------------------------------------------
# a7-a10: GLR and GTV operators
# ---------------------------------------------------------------------------
def glr_apply(x5: Tensor, wgt: Tensor, k: Tensor) -> Tensor:
    """GLRFast.forward: S^T (I - W) S x (REF:218-237)."""
    b, g, f, h, w = x5.shape
    s = stats_conv(x5, k)
    nb = gather_neighbors(s.reshape(b, g * f, h, w)).view(b, g, f, 4, h, w)
    ws = torch.einsum("bgfehw,bgehw->bgfhw", nb, wgt)
    return stats_conv_t(s - ws, k)


def gtv_C(x5: Tensor, wgt: Tensor, k: Tensor) -> Tensor:
    """GTVFast.op_C: E_e = w_e*Sx - w_e*(Sx)[clamp(p+delta_e)] -> [B,G,F,4,H,W] (REF:452-467)."""
    b, g, f, h, w = x5.shape
    s = stats_conv(x5, k)
    nb = gather_neighbors(s.reshape(b, g * f, h, w)).view(b, g, f, 4, h, w)
    we = wgt[:, :, None]
    return s[:, :, :, None] * we - nb * we


def gtv_Ct(e6: Tensor, wgt: Tensor, k: Tensor) -> Tensor:
    """GTVFast.op_C_transpose (REF:469-516).

    z_e = w_e * E_e; o(p) = sum_e z_e(p); then each z_e(p) is subtracted at
    p + delta_e inside a replicate-padded frame and the frame is cropped, so
    scatters landing outside the image are dropped; finally S^T.
    """
    b, g, f, ne, h, w = e6.shape
    z = e6 * wgt[:, :, None]
    o = z.sum(dim=3)
    ph, pw = PAD_HW
    frame = Fn.pad(o.reshape(b, g * f, h, w), (pw, pw, ph, ph), mode="replicate").view(
        b, g, f, h + 2 * ph, w + 2 * pw)
    for e, (dy, dx) in enumerate(EDGE_DELTA):
        sl = (slice(None), slice(None), slice(None),
              slice(ph + dy, ph + dy + h), slice(pw + dx, pw + dx + w))
        frame[sl] = frame[sl] - z[:, :, :, e]
    o = frame[:, :, :, ph:ph + h, pw:pw + w]
    return stats_conv_t(o, k)


def gtv_apply(x5: Tensor, wgt: Tensor, k: Tensor) -> Tensor:
    """GTVFast.forward: C^T C x (REF:518-523)."""
    return gtv_Ct(gtv_C(x5, wgt, k), wgt, k)


def soft_threshold(d: Tensor, gamma: Tensor) -> Tensor:
    """sign(d)*max(|d|-gamma, 0) written as the reference's two wheres (REF:684-704)."""
    gm = gamma[None, :, None, None, None, None]
    lo = torch.where(d < -gm, d + gm, 0.0)
    hi = torch.where(d > gm, d - gm, 0.0)
    return lo + hi


# ---------------------------------------------------------------------------
# 2x2 mean pool D and its transpose U (REF:613, :662-665, :676-679)
# ---------------------------------------------------------------------------
def pool2(x4: Tensor) -> Tensor:
    c = x4.shape[1]
    k = torch.full((c, 1, 2, 2), 0.25, dtype=x4.dtype)
    return Fn.conv2d(x4, k, stride=2, groups=c)


def unpool2(x4: Tensor) -> Tensor:
    c = x4.shape[1]
    k = torch.full((c, 1, 2, 2), 0.25, dtype=x4.dtype)
    return Fn.conv_transpose2d(x4, k, stride=2, groups=c)


# ---------------------------------------------------------------------------
# a11-a17: the MixtureGTVGLR solver
# ---------------------------------------------------------------------------
class _Graphs:
    """Edge weights + stencils of the four graph operators of one block."""

    def __init__(self, p: Params, f0: Tensor, f1: Tensor, g: int, nf: int):
        b, _, h, w = f0.shape
        c = g * nf
        ftv0, fgl0 = f0.chunk(2, dim=1)  # REF:714 first half GTV, second half GLR
        ftv1, fgl1 = f1.chunk(2, dim=1)  # REF:726
        h1, w1 = f1.shape[-2:]
        self.wG0, self.dG0 = edge_weights(ftv0.reshape(b, g, nf, h, w), p["GTVmodule00.multiM"])
        self.wL0, self.dL0 = edge_weights(fgl0.reshape(b, g, nf, h, w), p["GLRmodule00.multiM"])
        self.wG1, self.dG1 = edge_weights(ftv1.reshape(b, g, nf, h1, w1), p["GTVmodule01.multiM"])
        self.wL1, self.dL1 = edge_weights(fgl1.reshape(b, g, nf, h1, w1), p["GLRmodule01.multiM"])
        self.kG0 = stats_kernel(p, "GTVmodule00.")
        self.kL0 = stats_kernel(p, "GLRmodule00.")
        self.kG1 = stats_kernel(p, "GTVmodule01.")
        self.kL1 = stats_kernel(p, "GLRmodule01.")
        self.mu0 = torch.exp(p["muys00"])
        self.mu1 = torch.exp(p["muys01"])
        self.ro0 = torch.exp(p["ro00"])
        self.ro1 = torch.exp(p["ro01"])
        self.ga0 = torch.exp(p["gamma00"])
        self.ga1 = torch.exp(p["gamma01"])


def _scale(x5: Tensor, v: Tensor) -> Tensor:
    return x5 * v[None, :, None, None, None]


def system_operator(x5: Tensor, gr: _Graphs) -> Tensor:
    """A x = x + mu0 L0 x + ro0 G0 x + U(mu1 L1 D x + ro1 G1 D x) (REF:642-682)."""
    b, g, f, h, w = x5.shape
    out = x5 + _scale(glr_apply(x5, gr.wL0, gr.kL0), gr.mu0) + _scale(gtv_apply(x5, gr.wG0, gr.kG0), gr.ro0)
    xd = pool2(x5.reshape(b, g * f, h, w)).view(b, g, f, h // 2, w // 2)
    t = (_scale(glr_apply(xd, gr.wL1, gr.kL1), gr.mu1)
         + _scale(gtv_apply(xd, gr.wG1, gr.kG1), gr.ro1))
    return out + unpool2(t.reshape(b, g * f, h // 2, w // 2)).view(b, g, f, h, w)


def _gtv_rhs(y5: Tensor, x5: Tensor, gr: _Graphs, prox: bool) -> Tensor:
    """b = y + ro0 C0^T phi(C0 x) + ro1 U(C1^T phi(C1 D x)).

    prox=False is the rhs of REF:738-749 (x = y, phi = identity);
    prox=True is the GTV proximal rhs of REF:757-781 (phi(t) = eps - (t - eps),
    eps = soft_threshold(t, gamma)).
    """
    b, g, f, h, w = x5.shape
    t0 = gtv_C(x5, gr.wG0, gr.kG0)
    xd = pool2(x5.reshape(b, g * f, h, w)).view(b, g, f, h // 2, w // 2)
    t1 = gtv_C(xd, gr.wG1, gr.kG1)
    if prox:
        e0 = soft_threshold(t0, gr.ga0)
        e1 = soft_threshold(t1, gr.ga1)
        t0 = e0 - (t0 - e0)
        t1 = e1 - (t1 - e1)
    r = y5 + gtv_Ct(t0, gr.wG0, gr.kG0) * gr.ro0[None, :, None, None, None]
    u = unpool2(gtv_Ct(t1, gr.wG1, gr.kG1).reshape(b, g * f, h // 2, w // 2)).view(b, g, f, h, w)
    return r + u * gr.ro1[None, :, None, None, None]


def mixture_solve(y4: Tensor, p: Params, f0: Tensor, f1: Tensor, n_graphs: int,
                  n_stages: Optional[int] = None) -> Tensor:
    """Unrolled solver of MixtureGTVGLR.forward given its feature maps (REF:707-811).

    Stage recurrence (a17): x0 = b_A; x1 = x0 + a0 (b_A - A x0); prox -> b_B;
    r_k = b_B - A x_k; u_1 = r_1; u_k = r_k + beta_k u_{k-1} (k >= 2);
    x_{k+1} = x_k + alpha_k u_k; output x_S.  S = alphaCGD.shape[0] unless given.
    """
    b, c, h, w = y4.shape
    g = n_graphs
    nf = c // g
    alpha, beta = p["alphaCGD"], p["betaCGD"]
    s_count = alpha.shape[0] if n_stages is None else n_stages
    gr = _Graphs(p, f0, f1, g, nf)
    y5 = y4.reshape(b, g, nf, h, w)
    b_a = _gtv_rhs(y5, y5, gr, prox=False)
    x = b_a
    x = x + alpha[0][None, :, None, None, None] * (b_a - system_operator(x, gr))
    if s_count == 1:
        return x.reshape(b, c, h, w)
    b_b = _gtv_rhs(y5, x, gr, prox=True)
    u = None
    for k in range(1, s_count):
        r = b_b - system_operator(x, gr)
        u = r if u is None else r + beta[k][None, :, None, None, None] * u
        x = x + alpha[k][None, :, None, None, None] * u
    return x.reshape(b, c, h, w)


# ---------------------------------------------------------------------------
# Feature extractors
# ---------------------------------------------------------------------------
def conv1x1(x: Tensor, wgt: Tensor, groups: int = 1) -> Tensor:
    return Fn.conv2d(x, wgt, groups=groups)


def features_v1(y4: Tensor, p: Params) -> Tuple[Tensor, Tensor]:
    """v1.0 feature convs: 1x1 C->2C; 2x2/s2 C->C then 1x1 C->2C (REF:556-566, :593-612)."""
    f0 = Fn.conv2d(y4, p["patchs_features_extraction00.0.weight"])
    f1 = Fn.conv2d(y4, p["patchs_features_extraction01.0.weight"], stride=2)
    f1 = Fn.conv2d(f1, p["patchs_features_extraction01.1.weight"])
    return f0, f1


def custom_layer_norm(x: Tensor, p: Params, prefix: str, nsub: int) -> Tensor:
    """Per-pixel channel-group variance normalisation + depthwise 1x1 scale (REF:911-925)."""
    b, c, h, w = x.shape
    xs = x.reshape(b, nsub, c // nsub, h, w)
    var = xs.var(dim=2, keepdim=True, correction=1)
    xs = xs / torch.sqrt(var + 1e-5)
    return Fn.conv2d(xs.reshape(b, c, h, w), p[prefix + "weighted_transform.weight"], groups=c)


def local_nonlinear_block(x: Tensor, p: Params, prefix: str, nsub: int = 1) -> Tensor:
    """LocalNonLinearBlock: sw0*x + sw1*GatedLinear(LayerNorm(x)) (REF:929-964)."""
    n = custom_layer_norm(x, p, prefix + "norm.", nsub)
    ll = prefix + "local_linear."
    hcat = Fn.conv2d(n, p[ll + "channels_linear_op.weight"], groups=nsub)
    c2 = hcat.shape[1]
    hp = Fn.pad(hcat, (1, 1, 1, 1), mode="replicate")
    hcat = Fn.conv2d(hp, p[ll + "channels_local_linear_op.weight"], groups=c2)
    mask, val = hcat.chunk(2, dim=1)
    gated = torch.sigmoid(mask) * mask * val
    o = Fn.conv2d(gated, p[ll + "project_out.weight"], groups=nsub)
    sw = p[prefix + "skip_weight"]
    return sw[0] * x + sw[1] * o


def features_v13(y4: Tensor, p: Params) -> Tuple[Tensor, Tensor]:
    """Image-domain feature CNN: 3 LocalNonLinearBlocks + 1x1 per scale (REF13:612-637, :664-698)."""
    f0 = y4
    for i in range(3):
        f0 = local_nonlinear_block(f0, p, f"patchs_features_extraction00.{i}.")
    f0 = Fn.conv2d(f0, p["patchs_features_extraction00.3.weight"])
    f1 = Fn.conv2d(y4, p["patchs_features_extraction01.0.weight"], stride=2)
    for i in range(1, 4):
        f1 = local_nonlinear_block(f1, p, f"patchs_features_extraction01.{i}.")
    f1 = Fn.conv2d(f1, p["patchs_features_extraction01.4.weight"])
    return f0, f1


def mixture_glr_forward(y4: Tensor, p: Params, n_graphs: int, n_stages: Optional[int] = None) -> Tensor:
    """GLR-only single-scale MixtureGLR.forward of lib/model_GLR_GTV_deep_v10.py:241-335 (REF10).

    features = 1x1 conv C->C (REF10:270-281); one GLR graph (REF10:302-305); A x = x + mu L x with
    mu = muys00 used linearly (REF10:283-286, :296-305).  Recurrence (REF10:313-328):
    u_0 = r_0 = y - A y, x_1 = y + a_0 u_0;  u_k = (y - A x_k) + b_k u_{k-1}, x_{k+1} = x_k + a_k u_k.
    S = alphaCGD.shape[0] (3 in the reference) unless given.
    """
    b, c, h, w = y4.shape
    g = n_graphs
    nf = c // g
    feat = Fn.conv2d(y4, p["patchs_features_extraction.0.weight"])
    wgt, _ = edge_weights(feat.reshape(b, g, nf, h, w), p["GLRmodule00.multiM"])
    k = stats_kernel(p, "GLRmodule00.")
    mu = p["muys00"]
    alpha, beta = p["alphaCGD"], p["betaCGD"]
    s_count = alpha.shape[0] if n_stages is None else n_stages
    y5 = y4.reshape(b, g, nf, h, w)

    def system(x5):
        return x5 + _scale(glr_apply(x5, wgt, k), mu)

    u = y5 - system(y5)
    x = y5 + _scale(u, alpha[0])
    for i in range(1, s_count):
        u = (y5 - system(x)) + _scale(u, beta[i])
        x = x + _scale(u, alpha[i])
    return x.reshape(b, c, h, w)


def multiscale_glr_forward(y4: Tensor, p: Params, n_graphs: int, n_stages: Optional[int] = None) -> Tensor:
    """Two-scale GLR-only solver of config C2 (irdu_amd.MultiScaleMixtureGLR), composed from the
    pinned ops above.  No literal reference instance exists (SURVEY.md §8d "GLR-only, v10
    pattern, 2 scales"): the operator is REF:642-682 with its GTV / ro terms removed,
        A x = x + e^{mu0} L0 x + U(e^{mu1} L1 D x),
    features 1x1 C->C at full resolution (REF10:270-281) and 2x2/s2 + 1x1 at half resolution
    (REF:593-612), and the recurrence is REF10:313-328 with b = y.
    """
    b, c, h, w = y4.shape
    g = n_graphs
    nf = c // g
    f0 = Fn.conv2d(y4, p["patchs_features_extraction00.0.weight"])
    f1 = Fn.conv2d(Fn.conv2d(y4, p["patchs_features_extraction01.0.weight"], stride=2),
                   p["patchs_features_extraction01.1.weight"])
    w0, _ = edge_weights(f0.reshape(b, g, nf, h, w), p["GLRmodule00.multiM"])
    w1, _ = edge_weights(f1.reshape(b, g, nf, h // 2, w // 2), p["GLRmodule01.multiM"])
    k0, k1 = stats_kernel(p, "GLRmodule00."), stats_kernel(p, "GLRmodule01.")
    mu0, mu1 = torch.exp(p["muys00"]), torch.exp(p["muys01"])
    alpha, beta = p["alphaCGD"], p["betaCGD"]
    s_count = alpha.shape[0] if n_stages is None else n_stages
    y5 = y4.reshape(b, g, nf, h, w)

    def system(x5):
        xd = pool2(x5.reshape(b, c, h, w)).view(b, g, nf, h // 2, w // 2)
        t = _scale(glr_apply(xd, w1, k1), mu1)
        return x5 + _scale(glr_apply(x5, w0, k0), mu0) + unpool2(t.reshape(b, c, h // 2, w // 2)).view(b, g, nf, h, w)

    u = y5 - system(y5)
    x = y5 + _scale(u, alpha[0])
    for i in range(1, s_count):
        u = (y5 - system(x)) + _scale(u, beta[i])
        x = x + _scale(u, alpha[i])
    return x.reshape(b, c, h, w)


def multiscale_glr_image_filter(img: Tensor, p: Params, n_graphs: int, n_stages: Optional[int] = None) -> Tensor:
    """Config C2 image filter: gray image replicated over G graphs -> two-scale GLR -> 1x1."""
    b, cin, h, w = img.shape
    x = img[:, None].repeat(1, n_graphs, 1, 1, 1).reshape(b, n_graphs * cin, h, w)
    y = multiscale_glr_forward(x, sub_params(p, "localfilter."), n_graphs, n_stages)
    return Fn.conv2d(y, p["linear_combination.weight"])


def glr_image_filter(img: Tensor, p: Params, n_graphs: int, n_stages: Optional[int] = None) -> Tensor:
    """Single-scale GLR image filter (config C1): image replicated over G graphs -> v10 MixtureGLR -> 1x1."""
    b, cin, h, w = img.shape
    x = img[:, None].repeat(1, n_graphs, 1, 1, 1).reshape(b, n_graphs * cin, h, w)
    y = mixture_glr_forward(x, sub_params(p, "localfilter."), n_graphs, n_stages)
    return Fn.conv2d(y, p["linear_combination.weight"])


def sub_params(p: Params, prefix: str) -> Params:
    n = len(prefix)
    return {k[n:]: v for k, v in p.items() if k.startswith(prefix)}


def mixture_forward(y4: Tensor, p: Params, n_graphs: int, variant: str = "v1",
                    n_stages: Optional[int] = None) -> Tensor:
    """MixtureGTVGLR.forward (REF:707-811; REF13:808-884 for variant 'v13')."""
    feat = features_v1 if variant == "v1" else features_v13
    f0, f1 = feat(y4, p)
    return mixture_solve(y4, p, f0, f1, n_graphs, n_stages)


def lowpass_block(x: Tensor, p: Params, n_graphs: int, n_stages: Optional[int] = None) -> Tensor:
    """LocalLowpassFilteringBlock: s0*x + s1*MixtureGTVGLR(x) (REF:967-988)."""
    y = mixture_forward(x, sub_params(p, "local_filter."), n_graphs, "v1", n_stages)
    sw = p["skip_weight"]
    return sw[0] * x + sw[1] * y


def multiscale_graph_filter(img: Tensor, p: Params, n_graphs: int,
                            n_stages: Optional[int] = None) -> Tensor:
    """v13_no_latent MultiScaleGraphFilter: replicate RGB over G graphs, filter, 1x1 (REF13:887-926)."""
    b, cin, h, w = img.shape
    x = img[:, None].repeat(1, n_graphs, 1, 1, 1).reshape(b, n_graphs * cin, h, w)
    y = mixture_forward(x, sub_params(p, "localfilter."), n_graphs, "v13", n_stages)
    return Fn.conv2d(y, p["linear_combination.weight"])


# ---------------------------------------------------------------------------
# v1.0 end-to-end model (encoder/decoder around the filter; REF:1028-1174)
# ---------------------------------------------------------------------------
def _blocks(x: Tensor, p: Params, prefix: str, n: int, nsub: int) -> Tensor:
    for i in range(n):
        x = local_nonlinear_block(x, p, f"{prefix}.{i}.", nsub)
    return x


def abstract_encode(img: Tensor, p: Params, num_blocks: Sequence[int], nsubnets: Sequence[int]):
    x = Fn.pad(img, (1, 1, 1, 1), mode="replicate")
    x = Fn.conv2d(x, p["patch_3x3_embeding.channels_local_linear_op01.weight"])
    e0 = _blocks(x, p, "encoder_scale_00", num_blocks[0], nsubnets[0])
    e1 = _blocks(Fn.conv2d(e0, p["down_sample_00_01.local_linear.weight"], stride=2, groups=nsubnets[0]),
                 p, "encoder_scale_01", num_blocks[1], nsubnets[1])
    e2 = _blocks(Fn.conv2d(e1, p["down_sample_01_02.local_linear.weight"], stride=2, groups=nsubnets[1]),
                 p, "encoder_scale_02", num_blocks[2], nsubnets[2])
    e3 = _blocks(Fn.conv2d(e2, p["down_sample_02_03.local_linear.weight"], stride=2, groups=nsubnets[2]),
                 p, "encoder_scale_03", num_blocks[3], nsubnets[3])
    return e0, e1, e2, e3


def abstract_filtering(coefs, p: Params, ngraphs: Sequence[int], n_stages: Optional[int] = None):
    return tuple(lowpass_block(c, sub_params(p, f"localfilter_scale_0{i}."), ngraphs[i], n_stages)
                 for i, c in enumerate(coefs))


def abstract_decode(coefs, p: Params, num_blocks: Sequence[int], num_blocks_out: int,
                    nsubnets: Sequence[int]) -> Tensor:
    e0, e1, e2, e3 = coefs
    d = Fn.conv_transpose2d(e3, p["up_sample_03_02.local_linear.weight"], stride=2, groups=nsubnets[3])
    d = Fn.conv2d(torch.cat([d, e2], 1), p["combine_channels_02.weight"], groups=nsubnets[2])
    d = _blocks(d, p, "decoder_scale_02", num_blocks[2], nsubnets[2])
    d = Fn.conv_transpose2d(d, p["up_sample_02_01.local_linear.weight"], stride=2, groups=nsubnets[2])
    d = Fn.conv2d(torch.cat([d, e1], 1), p["combine_channels_01.weight"], groups=nsubnets[1])
    d = _blocks(d, p, "decoder_scale_01", num_blocks[1], nsubnets[1])
    d = Fn.conv_transpose2d(d, p["up_sample_01_00.local_linear.weight"], stride=2, groups=nsubnets[1])
    d = Fn.conv2d(torch.cat([d, e0], 1), p["combine_channels_00.weight"], groups=nsubnets[0])
    d = _blocks(d, p, "decoder_scale_00", num_blocks[0], nsubnets[0])
    d = _blocks(d, p, "refining_block", num_blocks_out, nsubnets[0])
    return Fn.conv2d(d, p["linear_output.weight"])


def abstract_forward(img: Tensor, p: Params, ngraphs: Sequence[int], num_blocks: Sequence[int],
                     num_blocks_out: int, nsubnets: Sequence[int] = (1, 1, 1, 1),
                     n_stages: Optional[int] = None) -> Tensor:
    """AbtractMultiScaleGraphFilter.forward = decode(filtering(encode(img))) (REF:1168-1174)."""
    coefs = abstract_encode(img, p, num_blocks, nsubnets)
    coefs = abstract_filtering(coefs, p, ngraphs, n_stages)
    return abstract_decode(coefs, p, num_blocks, num_blocks_out, nsubnets)


# ---------------------------------------------------------------------------
# Evaluation helpers (scripts_v2/run_abtract_lightformer_GGTV_GGLR_sigma25.py:276-286)
# ---------------------------------------------------------------------------
def img_as_ubyte(x: Tensor) -> Tensor:
    """skimage.img_as_ubyte for float input in [0,1]: x*255 rounded half-to-even (np.rint)."""
    return torch.round(x.clamp(0.0, 1.0).double() * 255.0).to(torch.uint8)


def psnr_ubyte(restored: Tensor, clean: Tensor) -> float:
    """20 log10(255/sqrt(mse)) on uint8-quantised images, as the reference's eval loop."""
    r = img_as_ubyte(restored).double()
    t = torch.round(clean.double() * 255.0)  # reference clean images are uint8
    mse = float(((t - r) ** 2).mean())
    return 20.0 * math.log10(255.0 / math.sqrt(mse)) if mse > 0 else float("inf")
