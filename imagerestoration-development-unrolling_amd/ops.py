"""The HIP entry points as ``torch.library`` custom operators (namespace ``irdu``).

The reference calls ``model.compile()`` (scripts_v2/run_abtract_lightformer_GGTV_GGLR_sigma25.py:130).
Under ``torch.compile`` every graph-filter launch must be an opaque node: Dynamo may not trace
into the ctypes call, and Inductor must not try to generate code for it (on ROCm that would be
Triton, which this engine does not use).  Each op below wraps one ``kernels`` function (which
launches one libgrr.so entry point on the current stream) and registers a fake (meta)
implementation with the output shapes, so the compiled graph of a graph-filter forward holds
only these ops and views.

Call sites use the Python helpers at the bottom (same arguments as ``kernels``, with a graph
module in place of its stencil struct).  In eager mode they call ``kernels`` directly -- the
same HIP kernel, without a dispatcher round trip per launch; while Dynamo traces
(``torch.compiler.is_compiling()``) they emit the custom op instead.

Absent optional outputs are returned as 0-element tensors by the ops (schemas have no optional
returns) and mapped back to None by the helpers.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
from torch import Tensor
from torch.library import custom_op

from . import kernels as K
from ._native import Stencil

NS = "irdu"


def _st(p01: Optional[Tensor], p02a: Optional[Tensor], p02b: Optional[Tensor], p03: Optional[Tensor]) -> Stencil:
    if p01 is None:
        return K.NO_STENCIL
    ps = [p.contiguous() for p in (p01, p02a, p02b, p03)]
    K._check("stencil", *ps)
    return Stencil(*[p.data_ptr() for p in ps])


def _none0(t: Optional[Tensor], like: Tensor) -> Tensor:
    return t if t is not None else like.new_empty(0)


def _half(x: Tensor) -> Tensor:
    b, c, h, w = x.shape
    return x.new_empty((b, c, h // 2, w // 2))


# ---- feature CNN -----------------------------------------------------------------------
@custom_op(f"{NS}::conv1x1", mutates_args=())
def conv1x1_op(x: Tensor, weight: Tensor) -> Tensor:
    return K.conv1x1(x.contiguous(), weight.contiguous())


@conv1x1_op.register_fake
def _(x, weight):
    return x.new_empty((x.shape[0], weight.shape[0], x.shape[2], x.shape[3]))


def _fold(weight: Tensor, cin: int) -> Tensor:
    """2x2/s2 conv weights [M, R*cin, 2, 2] summed over the R input replicas -> [M, cin, 2, 2]."""
    m, c = weight.shape[:2]
    return weight.reshape(m, c // cin, cin, 2, 2).sum(1).contiguous()


@custom_op(f"{NS}::conv2x2s2", mutates_args=())
def conv2x2s2_op(x: Tensor, weight: Tensor, fold: bool) -> Tensor:
    """fold: x holds one copy of an input that the weights see replicated over their channels."""
    w = _fold(weight, x.shape[1]) if fold else weight.contiguous()
    return K.conv2x2s2(x.contiguous(), w)


@conv2x2s2_op.register_fake
def _(x, weight, fold):
    return x.new_empty((x.shape[0], weight.shape[0], x.shape[2] // 2, x.shape[3] // 2))


@custom_op(f"{NS}::lnb_forward", mutates_args=())
def lnb_forward_op(x: Tensor, ln_w: Tensor, w1: Tensor, wdw: Tensor, w2: Tensor, skip: Tensor) -> Tensor:
    return K.lnb_forward(x.contiguous(), ln_w.contiguous(), w1.contiguous(), wdw.contiguous(), w2.contiguous(),
                         skip.contiguous())


@lnb_forward_op.register_fake
def _(x, ln_w, w1, wdw, w2, skip):
    return torch.empty_like(x)


@custom_op(f"{NS}::lnb_forward_rep", mutates_args=())
def lnb_forward_rep_op(src: Tensor, x: Optional[Tensor], ln_w: Tensor, w1: Tensor, wdw: Tensor, w2: Tensor,
                       skip: Tensor) -> Tensor:
    return K.lnb_forward_rep(src.contiguous(), None if x is None else x.contiguous(), ln_w.contiguous(),
                             w1.contiguous(), wdw.contiguous(), w2.contiguous(), skip.contiguous())


@lnb_forward_rep_op.register_fake
def _(src, x, ln_w, w1, wdw, w2, skip):
    return src.new_empty((src.shape[0], ln_w.numel(), src.shape[2], src.shape[3]))


@custom_op(f"{NS}::lnb_forward_c8", mutates_args=())
def lnb_forward_c8_op(x: Tensor, c: int, ln_w: Tensor, w1: Tensor, wdw: Tensor, w2: Tensor, skip: Tensor,
                      in_c8: bool, out_c8: bool) -> Tensor:
    return K.lnb_forward_c8(x.contiguous(), c, ln_w.contiguous(), w1.contiguous(), wdw.contiguous(), w2.contiguous(),
                            skip.contiguous(), in_c8, out_c8)


@lnb_forward_c8_op.register_fake
def _(x, c, ln_w, w1, wdw, w2, skip, in_c8, out_c8):
    b, h, w = (x.shape[0], x.shape[2], x.shape[3])
    return x.new_empty(K.c8_shape(b, c, h, w) if out_c8 else (b, c, h, w))


@custom_op(f"{NS}::feature_edges", mutates_args=())
def feature_edges_op(x: Tensor, x_blocked: bool, weight: Tensor, n_graphs: int, n_fts: int, multiM_gtv: Tensor,
                     multiM_glr: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    return K.feature_edges(x.contiguous(), x_blocked, weight.contiguous(), n_graphs, n_fts, multiM_gtv.contiguous(),
                           multiM_glr.contiguous())


@feature_edges_op.register_fake
def _(x, x_blocked, weight, n_graphs, n_fts, multiM_gtv, multiM_glr):
    b, h, w = (x.shape[0], x.shape[2], x.shape[3])
    return (x.new_empty((b, n_graphs, 4, h, w)), x.new_empty((b, n_graphs, 2, h, w)),
            x.new_empty((b, n_graphs, 4, h, w)))


@custom_op(f"{NS}::repeat_graphs", mutates_args=())
def repeat_graphs_op(img: Tensor, n_graphs: int) -> Tensor:
    return K.repeat_graphs(img.contiguous(), n_graphs)


@repeat_graphs_op.register_fake
def _(img, n_graphs):
    b, c, h, w = img.shape
    return img.new_empty((b, n_graphs * c, h, w))


# ---- graph operators -------------------------------------------------------------------
@custom_op(f"{NS}::pool2", mutates_args=())
def pool2_op(x: Tensor) -> Tensor:
    return K.pool2(x.contiguous())


@pool2_op.register_fake
def _(x):
    return _half(x)


@custom_op(f"{NS}::edge_weights", mutates_args=())
def edge_weights_op(feat: Tensor, channel_offset: int, n_graphs: int, n_fts: int, multiM: Tensor,
                    with_degree: bool) -> Tuple[Tensor, Tensor]:
    w, deg = K.edge_weights(feat.contiguous(), channel_offset, n_graphs, n_fts, multiM.contiguous(), with_degree)
    return w, _none0(deg, w)


@edge_weights_op.register_fake
def _(feat, channel_offset, n_graphs, n_fts, multiM, with_degree):
    b, _, h, w = feat.shape
    return feat.new_empty((b, n_graphs, 4, h, w)), (feat.new_empty((b, n_graphs, h, w)) if with_degree
                                                    else feat.new_empty(0))


@custom_op(f"{NS}::edge_weights_block", mutates_args=())
def edge_weights_block_op(feat: Tensor, n_graphs: int, n_fts: int, multiM_gtv: Tensor,
                          multiM_glr: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    return K.edge_weights_block(feat.contiguous(), n_graphs, n_fts, multiM_gtv.contiguous(), multiM_glr.contiguous())


@edge_weights_block_op.register_fake
def _(feat, n_graphs, n_fts, multiM_gtv, multiM_glr):
    b, _, h, w = feat.shape
    return (feat.new_empty((b, n_graphs, 4, h, w)), feat.new_empty((b, n_graphs, 2, h, w)),
            feat.new_empty((b, n_graphs, 4, h, w)))


@custom_op(f"{NS}::gtv_pair_weights", mutates_args=())
def gtv_pair_weights_op(w: Tensor) -> Tensor:
    return K.gtv_pair_weights(w.contiguous())


@gtv_pair_weights_op.register_fake
def _(w):
    b, g, _, h, ww = w.shape
    return w.new_empty((b, g, 2, h, ww))


@custom_op(f"{NS}::system_half", mutates_args=())
def system_half_op(xd: Tensor, wL: Optional[Tensor], cG: Optional[Tensor],
                   sL01: Optional[Tensor], sL02a: Optional[Tensor], sL02b: Optional[Tensor], sL03: Optional[Tensor],
                   sG01: Optional[Tensor], sG02a: Optional[Tensor], sG02b: Optional[Tensor], sG03: Optional[Tensor],
                   log_mu: Optional[Tensor], log_ro: Optional[Tensor], n_graphs: int) -> Tensor:
    return K.system_half(xd.contiguous(), wL, cG, _st(sL01, sL02a, sL02b, sL03), _st(sG01, sG02a, sG02b, sG03),
                         log_mu, log_ro, n_graphs)


@system_half_op.register_fake
def _(xd, *args):
    return torch.empty_like(xd)


@custom_op(f"{NS}::gtv_rhs_half", mutates_args=())
def gtv_rhs_half_op(xd: Tensor, wG: Tensor, s01: Tensor, s02a: Tensor, s02b: Tensor, s03: Tensor, prox: bool,
                    log_gamma: Optional[Tensor], n_graphs: int) -> Tensor:
    return K.gtv_rhs_half(xd.contiguous(), wG.contiguous(), _st(s01, s02a, s02b, s03), prox, log_gamma, n_graphs)


@gtv_rhs_half_op.register_fake
def _(xd, *args):
    return torch.empty_like(xd)


@custom_op(f"{NS}::gtv_rhs_full", mutates_args=())
def gtv_rhs_full_op(x: Tensor, x_rep: bool, y: Tensor, y_rep: bool, wG: Tensor, s01: Tensor, s02a: Tensor,
                    s02b: Tensor, s03: Tensor, prox: bool, log_gamma: Optional[Tensor], log_ro0: Tensor,
                    t_half: Optional[Tensor], log_ro1: Optional[Tensor], n_graphs: int,
                    want_pool: bool) -> Tuple[Tensor, Tensor]:
    st = _st(s01, s02a, s02b, s03)
    if x_rep or y_rep:
        out, xd = K.gtv_rhs_full_rep(x.contiguous(), x_rep, y.contiguous(), y_rep, wG.contiguous(), st, prox,
                                     log_gamma, log_ro0, t_half, log_ro1, n_graphs, want_pool=want_pool)
    else:
        out, xd = K.gtv_rhs_full(x.contiguous(), y.contiguous(), wG.contiguous(), st, prox, log_gamma, log_ro0,
                                 t_half, log_ro1, n_graphs, want_pool=want_pool)
    return out, _none0(xd, out)


@gtv_rhs_full_op.register_fake
def _(x, x_rep, y, y_rep, wG, s01, s02a, s02b, s03, prox, log_gamma, log_ro0, t_half, log_ro1, n_graphs, want_pool):
    ref = y if not y_rep else x
    b, c, h, w = ref.shape
    if x_rep and y_rep:
        c = c * n_graphs
    out = ref.new_empty((b, c, h, w))
    return out, (_half(out) if want_pool else out.new_empty(0))


@custom_op(f"{NS}::system_step", mutates_args=())
def system_step_op(x: Tensor, rhs: Tensor, u_prev: Optional[Tensor], t_half: Optional[Tensor], wL: Optional[Tensor],
                   cG: Optional[Tensor],
                   sL01: Optional[Tensor], sL02a: Optional[Tensor], sL02b: Optional[Tensor], sL03: Optional[Tensor],
                   sG01: Optional[Tensor], sG02a: Optional[Tensor], sG02b: Optional[Tensor], sG03: Optional[Tensor],
                   log_mu0: Optional[Tensor], log_ro0: Optional[Tensor], alpha: Tensor, beta: Optional[Tensor],
                   n_graphs: int, want_u: bool, want_pool: bool, skip: Optional[Tensor],
                   y_skip: Optional[Tensor]) -> Tuple[Tensor, Tensor, Tensor]:
    xo, u, xd = K.system_step(x.contiguous(), rhs.contiguous(), u_prev, t_half, wL, cG,
                              _st(sL01, sL02a, sL02b, sL03), _st(sG01, sG02a, sG02b, sG03), log_mu0, log_ro0,
                              alpha.contiguous(), None if beta is None else beta.contiguous(), n_graphs, want_u,
                              want_pool, skip, y_skip)
    return xo, _none0(u, xo), _none0(xd, xo)


@system_step_op.register_fake
def _(x, rhs, u_prev, t_half, wL, cG, sL01, sL02a, sL02b, sL03, sG01, sG02a, sG02b, sG03, log_mu0, log_ro0, alpha,
      beta, n_graphs, want_u, want_pool, skip, y_skip):
    return (torch.empty_like(x), torch.empty_like(x) if want_u else x.new_empty(0),
            _half(x) if want_pool else x.new_empty(0))


@custom_op(f"{NS}::system_step2", mutates_args=())
def system_step2_op(x: Tensor, rhs: Tensor, u_prev: Optional[Tensor], xd: Tensor, wL0: Tensor, cG0: Tensor,
                    sL01: Tensor, sL02a: Tensor, sL02b: Tensor, sL03: Tensor,
                    sG01: Tensor, sG02a: Tensor, sG02b: Tensor, sG03: Tensor, log_mu0: Tensor, log_ro0: Tensor,
                    wL1: Tensor, cG1: Tensor, tL01: Tensor, tL02a: Tensor, tL02b: Tensor, tL03: Tensor,
                    tG01: Tensor, tG02a: Tensor, tG02b: Tensor, tG03: Tensor, log_mu1: Tensor, log_ro1: Tensor,
                    alpha_a: Tensor, beta_a: Optional[Tensor], alpha_b: Tensor, beta_b: Optional[Tensor],
                    n_graphs: int, want_u: bool, want_pool: bool, skip: Optional[Tensor],
                    y_skip: Optional[Tensor]) -> Tuple[Tensor, Tensor, Tensor]:
    c = lambda t: None if t is None else t.contiguous()
    xo, u, xd = K.system_step2(x.contiguous(), rhs.contiguous(), u_prev, xd.contiguous(), wL0, cG0,
                               _st(sL01, sL02a, sL02b, sL03), _st(sG01, sG02a, sG02b, sG03), log_mu0, log_ro0,
                               wL1, cG1, _st(tL01, tL02a, tL02b, tL03), _st(tG01, tG02a, tG02b, tG03), log_mu1, log_ro1,
                               c(alpha_a), c(beta_a), c(alpha_b), c(beta_b), n_graphs, want_u, want_pool, skip, y_skip)
    return xo, _none0(u, xo), _none0(xd, xo)


@system_step2_op.register_fake
def _(x, rhs, u_prev, xd, wL0, cG0, sL01, sL02a, sL02b, sL03, sG01, sG02a, sG02b, sG03, log_mu0, log_ro0,
      wL1, cG1, tL01, tL02a, tL02b, tL03, tG01, tG02a, tG02b, tG03, log_mu1, log_ro1, alpha_a, beta_a, alpha_b,
      beta_b, n_graphs, want_u, want_pool, skip, y_skip):
    return (torch.empty_like(x), torch.empty_like(x) if want_u else x.new_empty(0),
            _half(x) if want_pool else x.new_empty(0))


@custom_op(f"{NS}::system_first_pair", mutates_args=())
def system_first_pair_op(b_a: Tensor, xd_a: Tensor, y: Tensor, y_rep: bool, wL0: Tensor, cG0: Tensor, wG0: Tensor,
                         sL01: Tensor, sL02a: Tensor, sL02b: Tensor, sL03: Tensor,
                         sG01: Tensor, sG02a: Tensor, sG02b: Tensor, sG03: Tensor, log_mu0: Tensor, log_ro0: Tensor,
                         log_gamma0: Tensor, wL1: Tensor, cG1: Tensor, wG1: Tensor,
                         tL01: Tensor, tL02a: Tensor, tL02b: Tensor, tL03: Tensor,
                         tG01: Tensor, tG02a: Tensor, tG02b: Tensor, tG03: Tensor, log_mu1: Tensor, log_ro1: Tensor,
                         log_gamma1: Tensor, alpha0: Tensor, alpha1: Tensor,
                         n_graphs: int) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    c = lambda t: t.contiguous()  # noqa: E731
    return K.system_first_pair(c(b_a), c(xd_a), c(y), y_rep, c(wL0), c(cG0), c(wG0), _st(sL01, sL02a, sL02b, sL03),
                               _st(sG01, sG02a, sG02b, sG03), c(log_mu0), c(log_ro0), c(log_gamma0), c(wL1), c(cG1),
                               c(wG1), _st(tL01, tL02a, tL02b, tL03), _st(tG01, tG02a, tG02b, tG03), c(log_mu1),
                               c(log_ro1), c(log_gamma1), c(alpha0), c(alpha1), n_graphs)


@system_first_pair_op.register_fake
def _(b_a, xd_a, y, y_rep, *args):
    return torch.empty_like(b_a), torch.empty_like(b_a), torch.empty_like(b_a), _half(b_a)


@custom_op(f"{NS}::glr_stage", mutates_args=())
def glr_stage_op(x: Tensor, b: Tensor, u_prev: Optional[Tensor], wL: Tensor, s01: Tensor, s02a: Tensor, s02b: Tensor,
                 s03: Tensor, mu: Tensor, alpha: Tensor, beta: Optional[Tensor], n_graphs: int,
                 want_u: bool) -> Tuple[Tensor, Tensor]:
    xo, u = K.glr_stage(x.contiguous(), b.contiguous(), u_prev, wL.contiguous(), _st(s01, s02a, s02b, s03),
                        mu.contiguous(), alpha.contiguous(), None if beta is None else beta.contiguous(), n_graphs,
                        want_u=want_u)
    return xo, _none0(u, xo)


@glr_stage_op.register_fake
def _(x, b, u_prev, wL, s01, s02a, s02b, s03, mu, alpha, beta, n_graphs, want_u):
    return torch.empty_like(x), (torch.empty_like(x) if want_u else x.new_empty(0))


# ---- GLRFast / GTVFast sub-API -------------------------------------------------------------
@custom_op(f"{NS}::neighbor_gather", mutates_args=())
def neighbor_gather_op(x: Tensor) -> Tensor:
    return K.neighbor_gather(x.contiguous())


@neighbor_gather_op.register_fake
def _(x):
    b, c, h, w = x.shape
    return x.new_empty((b, c, 4, h, w))


@custom_op(f"{NS}::normalize_features", mutates_args=())
def normalize_features_op(f5: Tensor, multiM: Tensor) -> Tensor:
    return K.normalize_features(f5.contiguous(), multiM.contiguous())


@normalize_features_op.register_fake
def _(f5, multiM):
    b, g, f, h, w = f5.shape
    return f5.new_empty((b, g * f, h, w))


@custom_op(f"{NS}::stats_conv", mutates_args=())
def stats_conv_op(x5: Tensor, s01: Tensor, s02a: Tensor, s02b: Tensor, s03: Tensor, transpose: bool) -> Tensor:
    return K.stats_conv(x5.contiguous(), _st(s01, s02a, s02b, s03), transpose)


@stats_conv_op.register_fake
def _(x5, *args):
    return torch.empty_like(x5)


@custom_op(f"{NS}::glr_op_L_norm", mutates_args=())
def glr_op_L_norm_op(x5: Tensor, w: Tensor) -> Tensor:
    return K.glr_op_L_norm(x5.contiguous(), w.contiguous())


@glr_op_L_norm_op.register_fake
def _(x5, w):
    return torch.empty_like(x5)


@custom_op(f"{NS}::gtv_op_C", mutates_args=())
def gtv_op_C_op(x5: Tensor, w: Tensor, s01: Tensor, s02a: Tensor, s02b: Tensor, s03: Tensor) -> Tensor:
    return K.gtv_op_C(x5.contiguous(), w.contiguous(), _st(s01, s02a, s02b, s03))


@gtv_op_C_op.register_fake
def _(x5, w, *args):
    b, g, f, h, ww = x5.shape
    return x5.new_empty((b, g, f, 4, h, ww))


@custom_op(f"{NS}::gtv_op_C_transpose", mutates_args=())
def gtv_op_C_transpose_op(e6: Tensor, w: Tensor, s01: Tensor, s02a: Tensor, s02b: Tensor, s03: Tensor) -> Tensor:
    return K.gtv_op_C_transpose(e6.contiguous(), w.contiguous(), _st(s01, s02a, s02b, s03))


@gtv_op_C_transpose_op.register_fake
def _(e6, w, *args):
    b, g, f, _, h, ww = e6.shape
    return e6.new_empty((b, g, f, h, ww))


OPS = [conv1x1_op, conv2x2s2_op, lnb_forward_op, lnb_forward_rep_op, repeat_graphs_op, pool2_op, edge_weights_op,
       edge_weights_block_op, gtv_pair_weights_op, system_half_op, gtv_rhs_half_op, gtv_rhs_full_op, system_step_op,
       system_step2_op, system_first_pair_op, glr_stage_op, neighbor_gather_op, normalize_features_op, stats_conv_op, glr_op_L_norm_op, gtv_op_C_op,
       gtv_op_C_transpose_op]


# =========================================================================================
# Call-site helpers: kernels' signatures, a GLRFast/GTVFast module (or None) for a stencil.
# =========================================================================================
def _tracing() -> bool:
    return torch.compiler.is_compiling()


def _sp(mod) -> List[Optional[Tensor]]:
    if mod is None:
        return [None, None, None, None]
    return [mod.stats_kernel_p01, mod.stats_kernel_p02a, mod.stats_kernel_p02b, mod.stats_kernel_p03]


def _opt(t: Tensor) -> Optional[Tensor]:
    return t if t.numel() else None


def conv1x1(x, weight):
    return torch.ops.irdu.conv1x1(x, weight) if _tracing() else K.conv1x1(x, weight)


def conv2x2s2(x, weight, fold=False):
    """fold: x is the un-replicated [B, cin, H, W] input of a conv whose input replicates it over its
    channels; the conv then equals the conv of x with the weights summed over the replicas."""
    if _tracing():
        return torch.ops.irdu.conv2x2s2(x, weight, fold)
    return K.conv2x2s2(x, _fold(weight, x.shape[1]) if fold else weight)


def lnb_forward(x, ln_w, w1, wdw, w2, skip):
    if _tracing():
        return torch.ops.irdu.lnb_forward(x, ln_w, w1, wdw, w2, skip)
    return K.lnb_forward(x, ln_w, w1, wdw, w2, skip)


def lnb_forward_rep(src, x, ln_w, w1, wdw, w2, skip):
    if _tracing():
        return torch.ops.irdu.lnb_forward_rep(src, x, ln_w, w1, wdw, w2, skip)
    return K.lnb_forward_rep(src, x, ln_w, w1, wdw, w2, skip)


def lnb_forward_c8(x, c, ln_w, w1, wdw, w2, skip, in_c8, out_c8):
    if _tracing():
        return torch.ops.irdu.lnb_forward_c8(x, c, ln_w, w1, wdw, w2, skip, in_c8, out_c8)
    return K.lnb_forward_c8(x, c, ln_w, w1, wdw, w2, skip, in_c8, out_c8)


def feature_edges(x, x_blocked, weight, n_graphs, n_fts, multiM_gtv, multiM_glr):
    if _tracing():
        return torch.ops.irdu.feature_edges(x, x_blocked, weight, n_graphs, n_fts, multiM_gtv, multiM_glr)
    return K.feature_edges(x, x_blocked, weight, n_graphs, n_fts, multiM_gtv, multiM_glr)


def repeat_graphs(img, n_graphs):
    return torch.ops.irdu.repeat_graphs(img, n_graphs) if _tracing() else K.repeat_graphs(img, n_graphs)


def pool2(x):
    return torch.ops.irdu.pool2(x) if _tracing() else K.pool2(x)


def edge_weights(feat, channel_offset, n_graphs, n_fts, multiM, with_degree=False):
    if _tracing():
        w, deg = torch.ops.irdu.edge_weights(feat, channel_offset, n_graphs, n_fts, multiM, with_degree)
        return w, _opt(deg)
    return K.edge_weights(feat, channel_offset, n_graphs, n_fts, multiM, with_degree)


def edge_weights_block(feat, n_graphs, n_fts, multiM_gtv, multiM_glr):
    if _tracing():
        return torch.ops.irdu.edge_weights_block(feat, n_graphs, n_fts, multiM_gtv, multiM_glr)
    return K.edge_weights_block(feat, n_graphs, n_fts, multiM_gtv, multiM_glr)


def gtv_pair_weights(w):
    return torch.ops.irdu.gtv_pair_weights(w) if _tracing() else K.gtv_pair_weights(w)


def system_half(xd, wL, cG, modL, modG, log_mu, log_ro, n_graphs):
    if _tracing():
        return torch.ops.irdu.system_half(xd, wL, cG, *_sp(modL), *_sp(modG), log_mu, log_ro, n_graphs)
    return K.system_half(xd, wL, cG, K.stencil(modL) if modL is not None else K.NO_STENCIL,
                         K.stencil(modG) if modG is not None else K.NO_STENCIL, log_mu, log_ro, n_graphs)


def gtv_rhs_half(xd, wG, modG, prox, log_gamma, n_graphs):
    if _tracing():
        return torch.ops.irdu.gtv_rhs_half(xd, wG, *_sp(modG), prox, log_gamma, n_graphs)
    return K.gtv_rhs_half(xd, wG, K.stencil(modG), prox, log_gamma, n_graphs)


def gtv_rhs_full(x, x_rep, y, y_rep, wG, modG, prox, log_gamma, log_ro0, t_half, log_ro1, n_graphs, want_pool=False):
    """grr_gtv_rhs_full(_rep): x / y given un-replicated when x_rep / y_rep."""
    if _tracing():
        out, xd = torch.ops.irdu.gtv_rhs_full(x, x_rep, y, y_rep, wG, *_sp(modG), prox, log_gamma, log_ro0, t_half,
                                              log_ro1, n_graphs, want_pool)
        return out, _opt(xd)
    if x_rep or y_rep:
        return K.gtv_rhs_full_rep(x, x_rep, y, y_rep, wG, K.stencil(modG), prox, log_gamma, log_ro0, t_half, log_ro1,
                                  n_graphs, want_pool=want_pool)
    return K.gtv_rhs_full(x, y, wG, K.stencil(modG), prox, log_gamma, log_ro0, t_half, log_ro1, n_graphs,
                          want_pool=want_pool)


def system_step(x, rhs, u_prev, t_half, wL, cG, modL, modG, log_mu0, log_ro0, alpha, beta, n_graphs, want_u,
                want_pool, skip=None, y_skip=None, u_out=None):
    """kernels.system_step; ``u_out`` (in-place direction reuse) applies to eager calls only (the
    custom op is functional)."""
    if _tracing():
        xo, u, xd = torch.ops.irdu.system_step(x, rhs, u_prev, t_half, wL, cG, *_sp(modL), *_sp(modG), log_mu0,
                                               log_ro0, alpha, beta, n_graphs, want_u, want_pool, skip, y_skip)
        return xo, _opt(u), _opt(xd)
    return K.system_step(x, rhs, u_prev, t_half, wL, cG, K.stencil(modL) if modL is not None else K.NO_STENCIL,
                         K.stencil(modG) if modG is not None else K.NO_STENCIL, log_mu0, log_ro0, alpha, beta,
                         n_graphs, want_u, want_pool, skip=skip, y_skip=y_skip, u_out=u_out)


def system_step2(x, rhs, u_prev, xd, wL0, cG0, modL0, modG0, log_mu0, log_ro0, wL1, cG1, modL1, modG1,
                 log_mu1, log_ro1, alpha_a, beta_a, alpha_b, beta_b, n_graphs, want_u, want_pool, skip=None,
                 y_skip=None, u_out=None):
    """kernels.system_step2 (stages k, k+1 in one pass, both half levels inside; xd = D x_k);
    ``u_out`` must not be u_prev (eager only)."""
    if _tracing():
        xo, u, xd = torch.ops.irdu.system_step2(x, rhs, u_prev, xd, wL0, cG0, *_sp(modL0), *_sp(modG0), log_mu0,
                                                log_ro0, wL1, cG1, *_sp(modL1), *_sp(modG1), log_mu1, log_ro1,
                                                alpha_a, beta_a, alpha_b, beta_b, n_graphs, want_u, want_pool, skip,
                                                y_skip)
        return xo, _opt(u), _opt(xd)
    return K.system_step2(x, rhs, u_prev, xd, wL0, cG0, K.stencil(modL0), K.stencil(modG0), log_mu0, log_ro0,
                          wL1, cG1, K.stencil(modL1), K.stencil(modG1), log_mu1, log_ro1, alpha_a, beta_a, alpha_b,
                          beta_b, n_graphs, want_u, want_pool, skip=skip, y_skip=y_skip, u_out=u_out)


def system_first_pair(b_a, xd_a, y, y_rep, wL0, cG0, wG0, modL0, modG0, log_mu0, log_ro0, log_gamma0, wL1, cG1, wG1,
                      modL1, modG1, log_mu1, log_ro1, log_gamma1, alpha0, alpha1, n_graphs):
    """kernels.system_first_pair (stage 0, right-hand side B, stage 1 in one pass; xd_a = D b_A).
    Returns (b_B, x_2, u_2, D x_2)."""
    if _tracing():
        return torch.ops.irdu.system_first_pair(b_a, xd_a, y, y_rep, wL0, cG0, wG0, *_sp(modL0), *_sp(modG0), log_mu0,
                                                log_ro0, log_gamma0, wL1, cG1, wG1, *_sp(modL1), *_sp(modG1), log_mu1,
                                                log_ro1, log_gamma1, alpha0, alpha1, n_graphs)
    return K.system_first_pair(b_a, xd_a, y, y_rep, wL0, cG0, wG0, K.stencil(modL0), K.stencil(modG0), log_mu0,
                               log_ro0, log_gamma0, wL1, cG1, wG1, K.stencil(modL1), K.stencil(modG1), log_mu1,
                               log_ro1, log_gamma1, alpha0, alpha1, n_graphs)


def first_pair_supported(x, n_graphs) -> bool:
    return K.STEP2 and K.first_pair_supported(x, n_graphs)


def step2_supported(x, n_graphs) -> bool:
    return K.STEP2 and K.step2_supported(x, n_graphs)


def glr_stage(x, b, u_prev, wL, modL, mu, alpha, beta, n_graphs, want_u=True, u_out=None):
    if _tracing():
        xo, u = torch.ops.irdu.glr_stage(x, b, u_prev, wL, *_sp(modL), mu, alpha, beta, n_graphs, want_u)
        return xo, _opt(u)
    return K.glr_stage(x, b, u_prev, wL, K.stencil(modL), mu, alpha, beta, n_graphs, want_u=want_u, u_out=u_out)


def neighbor_gather(x):
    return torch.ops.irdu.neighbor_gather(x) if _tracing() else K.neighbor_gather(x)


def normalize_features(f5, multiM):
    return torch.ops.irdu.normalize_features(f5, multiM) if _tracing() else K.normalize_features(f5, multiM)


def stats_conv(x5, mod, transpose):
    if _tracing():
        return torch.ops.irdu.stats_conv(x5, *_sp(mod), transpose)
    return K.stats_conv(x5, K.stencil(mod), transpose)


def glr_op_L_norm(x5, w):
    return torch.ops.irdu.glr_op_L_norm(x5, w) if _tracing() else K.glr_op_L_norm(x5, w)


def gtv_op_C(x5, w, mod):
    return torch.ops.irdu.gtv_op_C(x5, w, *_sp(mod)) if _tracing() else K.gtv_op_C(x5, w, K.stencil(mod))


def gtv_op_C_transpose(e6, w, mod):
    if _tracing():
        return torch.ops.irdu.gtv_op_C_transpose(e6, w, *_sp(mod))
    return K.gtv_op_C_transpose(e6, w, K.stencil(mod))
