"""Reverse pass of the graph filter on the HIP kernels (training, config C4).

The reference trains through PyTorch autograd over its op sequence
(REF = exploration/GGTV_GGLR_v1.0/deep_multiscale_GGLR_GGTV_v1x0.py).  Here the
forward runs the same fused HIP kernels as inference, keeping the iterates the
reverse sweep needs (x_k, u_k: 2 x S signal tensors), and the reverse sweep is
written out by hand on the adjoint kernels of graph_bwd.hip:

  solver      x_{k+1} = x_k + a_k u_k,  u_k = (b_B - A x_k) + b_k u_{k-1}     (REF:784-807)
              -> ga_k = <gx_{k+1}, u_k>_g,  gu_k = a_k gx_{k+1} + b_{k+1} gu_{k+1},
                 gb_k = <gu_k, u_{k-1}>_g,  gx_k = gx_{k+1} - A^T gu_k,  gb_B += gu_k
  stage 0     x_1 = b_A + a_0 r_0,  r_0 = b_A - A b_A                            (REF:751-753)
  rhs B       b_B = y + ro0 C0^T phi(C0 x_1) + ro1 U C1^T phi(C1 D x_1)          (REF:757-781)
  rhs A       b_A = y + ro0 G0 y + ro1 U G1 D y                                   (REF:736-749)
  operator    A = I + mu0 L0 + ro0 G0 + U (mu1 L1 + ro1 G1) D                     (REF:642-682)
  weights     pair weights -> raw w -> softmax / normalise / multiM -> features  (REF:146-175)

Every operator term  k * T(Z(P x))  (P = S, T = S^T, Z = I - W or the pair Laplacian)
is reversed in five passes: s = P x, a = T^* g, Z-reverse (z, Z^T a, weight gradient,
<a, z>), tap gradients of T and P, and x-gradient P^* (Z^T a).  All per-graph scalars
are differentiated as the reference stores them (logs of mu, ro, gamma).
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import os
import weakref

import torch

from . import kernels as K
from ._native import Stencil
from . import train_ops
from .train_ops import OpaqueFunction

Tensor = torch.Tensor

MODULES = ("GTVmodule00", "GLRmodule00", "GTVmodule01", "GLRmodule01")
STENCIL_PARAMS = ("stats_kernel_p01", "stats_kernel_p02a", "stats_kernel_p02b", "stats_kernel_p03")
SCALARS = ("muys00", "muys01", "ro00", "ro01", "gamma00", "gamma01", "alphaCGD", "betaCGD")
# order of the parameter tensors handed to _MixtureSolve.apply (MixtureGTVGLR attribute paths)
PARAM_NAMES = tuple(f"{m}.multiM" for m in MODULES) + tuple(
    f"{m}.{p}" for m in MODULES for p in STENCIL_PARAMS) + SCALARS


def solver_params(mod) -> List[Tensor]:
    out = []
    for name in PARAM_NAMES:
        obj = mod
        for part in name.split("."):
            obj = getattr(obj, part)
        out.append(obj)
    return out


FUSED_GATE_DW3 = True   # LNB reverse: gate + depthwise reverse in one row pass (False: two kernels; tests)
FUSED = True   # one-pass term reverses (grr_bwd_term_fused) where F has an instance; False: 5-pass path
PADJ2 = True   # the GLR and GTV terms' x-gradient passes of a level as one sweep (grr_bwd_padj2); False: two


def _use_fused(x: Tensor, n_graphs: int) -> bool:
    """One-pass term reverse: the row-streaming kernel (W <= 256, F <= 12) or the per-pixel one (F <= 4)."""
    f = x.shape[1] // n_graphs
    return FUSED and (f in K.FUSED_TERM_FTS or (K.TERM_ROWS and K.term_rows_ok(x.shape[3], f)))


# The x-gradient pass P*(v) inside the row-streaming term reverse (grr_bwd_term_fused_acc) wherever it
# takes the shape: v is never written and the padj2 / stencil pass that read it back is gone
TERM_ACC = True


def _acc_ok(mode: int, x: Tensor, g: Tensor, out: Tensor, n_graphs: int) -> bool:
    return TERM_ACC and FUSED and x.is_cuda and K.term_acc_ok(mode, x, n_graphs, g, out)


def glr_term_bwd(x: Tensor, g: Tensor, taps: Tensor, w: Tensor, scale: Tensor, coef: float, n_graphs: int,
                 out: Tensor, gw: Tensor, gscale: Optional[Tensor], gtaps: Tensor, defer: bool = False):
    """Reverse of the GLR term  scale[g] * T((I - W) P x)  (REF:218-237) contracted with coef * g:
    out += coef*scale * P*(I-W)^T T* g; gw, gtaps += coef*scale * d/d(.); gscale += coef * <g, T(I-W)Px>.
    defer (one-pass path only): return (v, coef*scale) and leave out += coef*scale P*(v) to the caller."""
    sc = scale * coef
    if not defer and _acc_ok(K.TERM_GLR, x, g, out, n_graphs):
        K.bwd_term_fused_acc(K.TERM_GLR, x, g, taps, w, None, sc, coef, out, gw, None, gscale, gtaps, n_graphs)
        return None
    if _use_fused(x, n_graphs):
        v = K.bwd_term_fused(K.TERM_GLR, x, g, taps, w, None, sc, coef, gw, None, gscale, gtaps, n_graphs)
        if defer:
            return v, sc
        K.bwd_stencil(v, taps, K.ST_P_ADJ, n_graphs, sc, out=out)
        return None
    s = K.bwd_stencil(x, taps, K.ST_P, n_graphs)
    a = K.bwd_stencil(g, taps, K.ST_T_ADJ, n_graphs)
    z, ap = K.bwd_glr(s, a, w, sc, coef, gw, gscale, n_graphs)
    del s, a
    K.bwd_tapgrad(g, z, K.ST_T, n_graphs, sc, gtaps)
    K.bwd_tapgrad(ap, x, K.ST_P, n_graphs, sc, gtaps)
    K.bwd_stencil(ap, taps, K.ST_P_ADJ, n_graphs, sc, out=out)


def gtv_term_bwd(x: Tensor, g: Tensor, taps: Tensor, c: Tensor, scale: Tensor, coef: float, n_graphs: int,
                 out: Tensor, gc: Tensor, gscale: Optional[Tensor], gtaps: Tensor, defer: bool = False):
    """Reverse of the linear GTV term  scale[g] * T(K_c P x)  (C^T C with pair weights, REF:452-523)."""
    sc = scale * coef
    if not defer and _acc_ok(K.TERM_PAIR, x, g, out, n_graphs):
        K.bwd_term_fused_acc(K.TERM_PAIR, x, g, taps, c, None, sc, coef, out, gc, None, gscale, gtaps, n_graphs)
        return None
    if _use_fused(x, n_graphs):
        v = K.bwd_term_fused(K.TERM_PAIR, x, g, taps, c, None, sc, coef, gc, None, gscale, gtaps, n_graphs)
        if defer:
            return v, sc
        K.bwd_stencil(v, taps, K.ST_P_ADJ, n_graphs, sc, out=out)
        return None
    s = K.bwd_stencil(x, taps, K.ST_P, n_graphs)
    a = K.bwd_stencil(g, taps, K.ST_T_ADJ, n_graphs)
    z, ap = K.bwd_pair(s, a, c, sc, coef, gc, gscale, n_graphs)
    del s, a
    K.bwd_tapgrad(g, z, K.ST_T, n_graphs, sc, gtaps)
    K.bwd_tapgrad(ap, x, K.ST_P, n_graphs, sc, gtaps)
    K.bwd_stencil(ap, taps, K.ST_P_ADJ, n_graphs, sc, out=out)


class _Level:
    """One resolution level of the operator: its graphs, stencils, scalars and gradient buffers."""

    def __init__(self, wL, cG, wG, stL, stG, log_mu, log_ro, log_gamma, g):
        self.wL, self.cG, self.wG = wL, cG, wG
        self.stL, self.stG = stL, stG                     # (p01, p02a, p02b, p03) tensors
        self.tapsL, self.tapsG = K.stencil_taps(*stL), K.stencil_taps(*stG)
        self.log_mu, self.log_ro, self.log_gamma = log_mu, log_ro, log_gamma
        self.mu, self.ro = torch.exp(log_mu), torch.exp(log_ro)
        self.g = g
        z = torch.zeros_like
        self.gwL, self.gcG, self.gwG = z(wL), z(cG), z(wG)
        self.gtapL, self.gtapG = z(self.tapsL), z(self.tapsG)
        self.gmu, self.gro, self.ggam = z(log_mu), z(log_ro), z(log_gamma)

    def terms_bwd(self, x: Tensor, g: Tensor, coef: float, out: Tensor, glr: bool = True,
                  defer: bool = False) -> Optional[tuple]:
        """out += coef * (mu L^T + ro G^T) g, and coef * d<g, mu L x + ro G x>/d(params) into the buffers.
        With both one-pass term reverses, the two x-gradient passes run as one sweep (grr_bwd_padj2);
        defer: that sweep's operands are returned instead (the next bwd_cg_glue applies them)."""
        acc = _acc_ok(K.TERM_PAIR, x, g, out, self.g) and (not glr or _acc_ok(K.TERM_GLR, x, g, out, self.g))
        if glr and PADJ2 and not acc and _use_fused(x, self.g) and K.padj2_ok(x):
            vl, scl = glr_term_bwd(x, g, self.tapsL, self.wL, self.mu, coef, self.g, out, self.gwL, self.gmu,
                                   self.gtapL, defer=True)
            vg, scg = gtv_term_bwd(x, g, self.tapsG, self.cG, self.ro, coef, self.g, out, self.gcG, self.gro,
                                   self.gtapG, defer=True)
            if defer:
                return (vl, self.tapsL, scl, vg, self.tapsG, scg)
            K.bwd_padj2(vl, self.tapsL, scl, vg, self.tapsG, scg, out, self.g)
            return None
        if glr:
            glr_term_bwd(x, g, self.tapsL, self.wL, self.mu, coef, self.g, out, self.gwL, self.gmu, self.gtapL)
        gtv_term_bwd(x, g, self.tapsG, self.cG, self.ro, coef, self.g, out, self.gcG, self.gro, self.gtapG)
        return None

    def prox_bwd(self, x: Tensor, g: Tensor, out: Tensor) -> None:
        """out += ro C^T-part reverse of the prox rhs term ro T(Ct phi(C P x)); parameter gradients."""
        G = self.g
        sc = self.ro
        if _acc_ok(K.TERM_PROX, x, g, out, G):
            K.bwd_term_fused_acc(K.TERM_PROX, x, g, self.tapsG, self.wG, self.log_gamma, sc, 1.0, out, self.gwG,
                                 self.ggam, self.gro, self.gtapG, G)
            return
        if _use_fused(x, G):
            v = K.bwd_term_fused(K.TERM_PROX, x, g, self.tapsG, self.wG, self.log_gamma, sc, 1.0, self.gwG,
                                 self.ggam, self.gro, self.gtapG, G)
            K.bwd_stencil(v, self.tapsG, K.ST_P_ADJ, G, sc, out=out)
            return
        s = K.bwd_stencil(x, self.tapsG, K.ST_P, G)
        a = K.bwd_stencil(g, self.tapsG, K.ST_T_ADJ, G)
        o, gs = K.bwd_prox(s, a, self.wG, self.log_gamma, sc, 1.0, self.gwG, self.ggam, self.gro, G)
        del s, a
        K.bwd_tapgrad(g, o, K.ST_T, G, sc, self.gtapG)
        K.bwd_tapgrad(gs, x, K.ST_P, G, sc, self.gtapG)
        K.bwd_stencil(gs, self.tapsG, K.ST_P_ADJ, G, sc, out=out)


# The half level's reverse runs on a second HIP stream beside the full level's (GRR_LEVEL_STREAMS=0: one
# stream): the two touch disjoint gradient buffers until U adds the half level's x-gradient, and the
# small launches of the deeper levels of the v1.0 model leave most of the GPU idle one at a time
LEVEL_STREAMS = os.environ.get("GRR_LEVEL_STREAMS", "1") == "1"
_LEVEL_SIDE = {}


def _level_side(dev: torch.device) -> "torch.cuda.Stream":
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    if key not in _LEVEL_SIDE:
        _LEVEL_SIDE[key] = torch.cuda.Stream(device=dev)
    return _LEVEL_SIDE[key]


# The half level's x-gradient of stage k's operator reverse is added by the next stage's glue pass
# (grr_bwd_cg_glue's gx_half: U folded into the pass that reads gx next) instead of its own
# unpool-accumulate pass (a read + write of the full-resolution gradient)
UNPOOL_GLUE = True
# ... and the full level's padj2 sweep of stage k likewise (grr_bwd_cg_glue's v1 / v2), where it runs
PADJ_GLUE = True
# The training forward keeps D x_k (its kernels form them anyway) for the reverse sweep's half level:
# no pool2 of the saved iterates there (C/4 floats per pixel per stage of extra saved memory)
SAVE_POOLED = os.environ.get("GRR_SAVE_POOLED", "1") == "1"
# ... and the glue pass that writes gu_k also writes D gu_k (grr_bwd_cg_glue_pool): no pool2 of gu_k
GLUE_POOL = os.environ.get("GRR_GLUE_POOL", "1") == "1"
# LNB / FFBlock reverse: the skip term (s0 gout, <gout, x>) inside the norm's reverse pass
LN_SKIP_FUSED = True


def _two_level(l0: _Level, l1: _Level, x: Tensor, g: Tensor, out: Tensor, fn,
               defer: bool = False, xd: Optional[Tensor] = None, gd: Optional[Tensor] = None) -> Optional[Tensor]:
    """Apply a per-level reverse at full resolution and, through D / U, at half resolution.
    defer: return the half level's x-gradient instead of adding U of it to out (the caller passes it
    to the next bwd_cg_glue).  xd, gd: D x saved by the forward, D g formed by the pass that wrote g
    (else pooled here)."""
    if LEVEL_STREAMS and x.is_cuda and not torch.compiler.is_compiling() \
            and not torch.cuda.is_current_stream_capturing():
        main = torch.cuda.current_stream(x.device)
        side = _level_side(x.device)
        side.wait_stream(main)                # x, g (and every buffer the half level accumulates into) ready
        with torch.cuda.stream(side):
            xd = K.pool2(x) if xd is None else xd
            gd = K.pool2(g) if gd is None else gd
            gxd = torch.zeros_like(xd)
            fn(l1, xd, gd, gxd)
        x.record_stream(side)
        g.record_stream(side)
        fn(l0, x, g, out)
        main.wait_stream(side)
        gxd.record_stream(main)
        if defer:
            return gxd
        K.bwd_unpool2_acc(gxd, out)           # D^T = U
        return None
    fn(l0, x, g, out)
    xd = K.pool2(x) if xd is None else xd          # half level sees D x; U^T = D
    gd = K.pool2(g) if gd is None else gd
    gxd = torch.zeros_like(xd)
    fn(l1, xd, gd, gxd)
    if defer:
        return gxd
    K.bwd_unpool2_acc(gxd, out)               # D^T = U
    return None


def cg_glue(gx: Tensor, u: Tensor, gu_next: Optional[Tensor], u_prev: Optional[Tensor], alpha: Tensor, beta: Tensor,
            gbb: Optional[Tensor], galpha: Tensor, gbeta: Tensor, k: int, g: int, owned: bool,
            gx_half: Optional[Tensor] = None, padj: Optional[tuple] = None, want_pool: bool = False):
    """Reverse of stage k's recurrence glue (x' = x + a_k u_k, u_k = r - A x + b_k u_{k-1}) without the
    operator term: returns (gu_k, gx' - gu_k), and D gu_k third when want_pool; ga_k, gb_k (when
    u_prev) and gbb accumulate.  owned: gx is this sweep's own buffer and is overwritten."""
    return K.bwd_cg_glue(gx, u, gu_next, u_prev, alpha[k].contiguous(),
                         beta[k + 1].contiguous() if gu_next is not None else None, gbb, galpha[k],
                         gbeta[k] if u_prev is not None else None, g, inplace=owned, gx_half=gx_half,
                         padj=padj, want_pool=want_pool)


def _stencil(t4) -> Stencil:
    return Stencil(*[t.data_ptr() for t in t4])


# Each differentiable HIP operation below is a pair of pure functions (forward -> outputs + the
# tensors the reverse needs; reverse -> input gradients) wrapped by train_ops.OpaqueFunction: a
# plain autograd.Function in eager mode, one opaque irdu:: custom op per direction under
# torch.compile.  `consts` carries the integer arguments (graph count, kind).

def _new(x: Tensor, *shape) -> Tensor:
    return x.new_empty(shape)


# ---- MixtureGTVGLR solve (REF:707-811) ----------------------------------------------------
def _mixture_fwd(consts, y: Tensor, f0: Tensor, f1: Tensor, *params: Tensor):
    p = dict(zip(PARAM_NAMES, params))
    g = consts[0]
    b, c, h, w = y.shape
    nf = c // g
    wG0, cG0, wL0 = K.edge_weights_block(f0, g, nf, p["GTVmodule00.multiM"], p["GLRmodule00.multiM"])
    wG1, cG1, wL1 = K.edge_weights_block(f1, g, nf, p["GTVmodule01.multiM"], p["GLRmodule01.multiM"])
    st = {m: tuple(p[f"{m}.{q}"] for q in STENCIL_PARAMS) for m in MODULES}
    sG0, sL0, sG1, sL1 = (_stencil(st[m]) for m in MODULES)
    mu0, mu1, ro0, ro1 = p["muys00"], p["muys01"], p["ro00"], p["ro01"]
    alpha, beta = p["alphaCGD"], p["betaCGD"]
    n_st = alpha.shape[0]

    keep = bool(consts[1])
    dy = K.pool2(y)
    t = K.gtv_rhs_half(dy, cG1, sG1, False, None, g)
    b_a, xd = K.gtv_rhs_full(y, y, cG0, sG0, False, None, ro0, t, ro1, g, want_pool=True)
    xds = [xd]
    t = K.system_half(xd, wL1, cG1, sL1, sG1, mu1, ro1, g)
    x, r0, xd = K.system_step(b_a, b_a, None, t, wL0, cG0, sL0, sG0, mu0, ro0, alpha[0], None, g,
                              want_u=True, want_pool=n_st > 1)
    xs, us = [b_a, x], [r0]
    if n_st > 1:
        xds.append(xd)
    if n_st > 1:
        t = K.gtv_rhs_half(xd, wG1, sG1, True, p["gamma01"], g)
        b_b, _ = K.gtv_rhs_full(x, y, wG0, sG0, True, p["gamma00"], ro0, t, ro1, g)
        u = None
        pair = K.STEP2 and K.step2_supported(x, g)
        k = 1
        while k < n_st:
            if pair and k + 1 < n_st:
                # stages k, k+1 in one pass; the middle iterate is written for the reverse sweep
                last = k + 1 == n_st - 1
                xm, um, x, u, xd, xdm = K.system_step2_train(x, b_b, u, xd, wL0, cG0, sL0, sG0, mu0, ro0, wL1, cG1,
                                                             sL1, sG1, mu1, ro1, alpha[k], beta[k] if k >= 2 else None,
                                                             alpha[k + 1], beta[k + 1], g, want_pool=not last,
                                                             want_mid_pool=keep)
                xs += [xm, x]
                us += [um, u]
                xds += [xdm, xd]
                k += 2
                continue
            last = k == n_st - 1
            t = K.system_half(xd, wL1, cG1, sL1, sG1, mu1, ro1, g)
            x, u, xd = K.system_step(x, b_b, u, t, wL0, cG0, sL0, sG0, mu0, ro0, alpha[k],
                                     beta[k] if k >= 2 else None, g, want_u=True, want_pool=not last)
            xs.append(x)
            us.append(u)
            xds.append(xd)
            k += 1
        del b_b
    # keep: D x_0 ... D x_{S-1} and D y, the half-level operands of the reverse sweep (no pool2 of them there)
    pooled = [*xds[:n_st], dy] if keep else []
    return [xs[-1]], [wG0, wL0, wG1, wL1, cG0, cG1, *xs[:-1], *us, *pooled]


def _mixture_fake(consts, y: Tensor, f0: Tensor, f1: Tensor, *params: Tensor):
    g = consts[0]
    b, c, h, w = y.shape
    n_st = dict(zip(PARAM_NAMES, params))["alphaCGD"].shape[0]
    e0, e1 = _new(y, b, g, 4, h, w), _new(y, b, g, 4, h // 2, w // 2)
    pooled = [_new(y, b, c, h // 2, w // 2) for _ in range(n_st + 1)] if consts[1] else []
    return [_new(y, b, c, h, w)], [e0, _new(y, b, g, 4, h, w), e1, _new(y, b, g, 4, h // 2, w // 2),
                                   _new(y, b, g, 2, h, w), _new(y, b, g, 2, h // 2, w // 2),
                                   *[_new(y, b, c, h, w) for _ in range(2 * n_st)], *pooled]


def _mixture_bwd(consts, inputs, outs, saved, gouts, needs):
    g = consts[0]
    y, f0, f1 = inputs[:3]
    params = inputs[3:]
    keep = bool(consts[1])
    n_st = (len(saved) - 6 - int(keep)) // (3 if keep else 2)
    wG0, wL0, wG1, wL1, cG0, cG1 = saved[:6]
    xs = saved[6:6 + n_st]          # x_0 = b_A, x_1, ..., x_{S-1}
    us = saved[6 + n_st:6 + 2 * n_st]   # r_0, u_1, ..., u_{S-1}
    # D x_0 ... D x_{S-1}, D y from the forward (keep), else pooled here
    xds = saved[6 + 2 * n_st:] if keep else [None] * (n_st + 1)
    p = dict(zip(PARAM_NAMES, params))
    c = y.shape[1]
    nf = c // g
    st = {m: tuple(p[f"{m}.{q}"] for q in STENCIL_PARAMS) for m in MODULES}
    l0 = _Level(wL0, cG0, wG0, st["GLRmodule00"], st["GTVmodule00"], p["muys00"], p["ro00"], p["gamma00"], g)
    l1 = _Level(wL1, cG1, wG1, st["GLRmodule01"], st["GTVmodule01"], p["muys01"], p["ro01"], p["gamma01"], g)
    alpha, beta = p["alphaCGD"], p["betaCGD"]
    galpha, gbeta = torch.zeros_like(alpha), torch.zeros_like(beta)

    def a_bwd(x, gg, coef, out, glr=True, defer=False, xd=None, gd=None):   # out += coef * (A - I)^T gg (+ params)
        # defer: the full level's padj2 operands and the half level's x-gradient are returned for the
        # next bwd_cg_glue instead of being added to out here
        pend = []

        def fn(lv, xx, g2, o):
            r = lv.terms_bwd(xx, g2, coef, o, glr, defer=defer and PADJ_GLUE and lv is l0)
            if r is not None:
                pend.append(r)
        gxh = _two_level(l0, l1, x, gg, out, fn, defer, xd, gd)
        return gxh, (pend[0] if pend else None)

    gx = gouts[0].contiguous()
    gy = torch.zeros_like(y)
    if n_st > 1:
        gbb = torch.zeros_like(y)
        gu_next, gxh, pj = None, None, None
        for k in range(n_st - 1, 0, -1):
            # ga_k, gu_k, gb_k, gb_B += gu_k, gx_{k+1} - gu_k in one pass (grr_bwd_cg_glue), with the
            # previous stage's full-level x-gradient pass and half-level x-gradient added on the way in
            pool = GLUE_POOL and K.glue_pool_ok(gx, us[k], gu_next, us[k - 1] if k >= 2 else None, gbb,
                                                *((pj[0], pj[3]) if pj is not None else ()), gx_half=gxh)
            gu, gx, *gud = cg_glue(gx, us[k], gu_next, us[k - 1] if k >= 2 else None, alpha, beta, gbb,
                                   galpha, gbeta, k, g, owned=k < n_st - 1, gx_half=gxh, padj=pj, want_pool=pool)
            gxh, pj = a_bwd(xs[k], gu, -1.0, gx, defer=UNPOOL_GLUE and k > 1, xd=xds[k],
                            gd=gud[0] if gud else None)                   #   - (A - I)^T gu
            del gud
            gu_next = gu
        # b_B = y + prox terms(x_1)
        K.bwd_lincomb(gbb, None, None, None, g, out=gy, accumulate=True)
        _two_level(l0, l1, xs[1], gbb, gx, lambda lv, xx, g2, o: lv.prox_bwd(xx, g2, o), xd=xds[1])
        del gbb
    # x_1 = b_A + alpha_0 r_0, r_0 = b_A - A b_A
    K.bwd_graph_dot(gx, us[0], galpha[0], g)
    ga = K.bwd_lincomb(gx, alpha[0], None, None, g)
    gba = gx.clone()
    a_bwd(xs[0], ga, -1.0, gba, xd=xds[0])                      # gx_1 - (A - I)^T (alpha_0 gx_1)
    del ga
    # b_A = y + ro0 G0 y + U ro1 G1 D y
    K.bwd_lincomb(gba, None, None, None, g, out=gy, accumulate=True)
    a_bwd(y, gba, 1.0, gy, glr=False, xd=xds[n_st])
    del gba

    # weights -> features
    K.bwd_pair_weights(wG0, l0.gcG, l0.gwG)
    K.bwd_pair_weights(wG1, l1.gcG, l1.gwG)
    gf0, gf1 = torch.empty_like(f0), torch.empty_like(f1)
    gM = {m: torch.zeros_like(p[f"{m}.multiM"]) for m in MODULES}
    K.bwd_edge_weights(f0, 0, g, nf, p["GTVmodule00.multiM"], wG0, l0.gwG, gf0, gM["GTVmodule00"])
    K.bwd_edge_weights(f0, c, g, nf, p["GLRmodule00.multiM"], wL0, l0.gwL, gf0, gM["GLRmodule00"])
    K.bwd_edge_weights(f1, 0, g, nf, p["GTVmodule01.multiM"], wG1, l1.gwG, gf1, gM["GTVmodule01"])
    K.bwd_edge_weights(f1, c, g, nf, p["GLRmodule01.multiM"], wL1, l1.gwL, gf1, gM["GLRmodule01"])

    grads = {f"{m}.multiM": gM[m] for m in MODULES}
    for m, gt in (("GTVmodule00", l0.gtapG), ("GLRmodule00", l0.gtapL),
                  ("GTVmodule01", l1.gtapG), ("GLRmodule01", l1.gtapL)):
        for q, gq in zip(STENCIL_PARAMS, K.stencil_taps_backward(gt)):
            grads[f"{m}.{q}"] = gq
    grads["muys00"], grads["muys01"] = l0.gmu * l0.mu, l1.gmu * l1.mu
    grads["ro00"], grads["ro01"] = l0.gro * l0.ro, l1.gro * l1.ro
    grads["gamma00"] = l0.ggam * torch.exp(l0.log_gamma)
    grads["gamma01"] = l1.ggam * torch.exp(l1.log_gamma)
    grads["alphaCGD"], grads["betaCGD"] = galpha, gbeta
    return (gy, gf0, gf1, *[grads[n] for n in PARAM_NAMES])


MIXTURE = OpaqueFunction("mixture_solve_train", 1, _mixture_fwd, _mixture_bwd, _mixture_fake)


def mixture_solve(mod, y: Tensor, f0: Tensor, f1: Tensor) -> Tensor:
    """Differentiable MixtureGTVGLR solve (features given); all work on the HIP kernels."""
    return MIXTURE([mod.n_graphs, int(SAVE_POOLED)], y, f0.contiguous(), f1.contiguous(), *solver_params(mod))


# ---- feature convolutions ----------------------------------------------------
# nn.Conv2d(K, M, 1, bias=False): forward and data gradient on the HIP GEMM; the weight gradient (a
# reduction over B*H*W) is grr_wgrad (fp32 MFMA partial tiles per pixel chunk, added in a fixed order)
def _conv1x1_fwd(consts, x: Tensor, weight: Tensor):
    return [K.conv1x1(x.contiguous(), weight.contiguous())], []


def _conv1x1_bwd(consts, inputs, outs, saved, gouts, needs):
    x, weight = inputs
    g = gouts[0].contiguous()
    m, k = weight.shape[:2]
    gx = K.conv1x1(g, weight.reshape(m, k).t().contiguous().view(k, m, 1, 1)) if needs[0] else None
    b = x.shape[0]
    gw = K.wgrad(g, x.contiguous())
    return gx, gw.view_as(weight)


def _conv1x1_fake(consts, x: Tensor, weight: Tensor):
    return [_new(x, x.shape[0], weight.shape[0], x.shape[2], x.shape[3])], []


CONV1X1 = OpaqueFunction("conv1x1_train", 1, _conv1x1_fwd, _conv1x1_bwd, _conv1x1_fake)


# nn.Conv2d(K, M, 2, stride=2, bias=False) (REF:593-602): HIP forward and data gradient, weight gradient
# on grr_wgrad over the 2x2 patches
def _conv2x2_fwd(consts, x: Tensor, weight: Tensor):
    return [K.conv2x2s2(x.contiguous(), weight.contiguous())], []


def _conv2x2_bwd(consts, inputs, outs, saved, gouts, needs):
    x, weight = inputs
    g = gouts[0].contiguous()
    b, k, h, w = x.shape
    m = weight.shape[0]
    gx = None
    if needs[0]:
        # one 4K-row GEMM (split-bf16 for M <= 128, fp32 MFMA above) + interleave (W % 4 == 0)
        if w % 4 == 0:
            gx = K.conv2x2s2_bwd_data_gemm(g, weight.contiguous(), h, w)
        else:
            gx = K.conv2x2s2_bwd_data(g, weight.contiguous(), h, w)
    # patch rows in the weight's (k, dy, dx) order: [B, 4K, H/2 * W/2]
    patches = x.reshape(b, k, h // 2, 2, w // 2, 2).permute(0, 1, 3, 5, 2, 4).reshape(b, k * 4, -1)
    gw = K.wgrad(g, patches)
    return gx, gw.view_as(weight)


def _conv2x2_fake(consts, x: Tensor, weight: Tensor):
    return [_new(x, x.shape[0], weight.shape[0], x.shape[2] // 2, x.shape[3] // 2)], []


CONV2X2S2 = OpaqueFunction("conv2x2s2_train", 1, _conv2x2_fwd, _conv2x2_bwd, _conv2x2_fake)


# img [B,Cin,H,W] -> [B,G*Cin,H,W] replicated over the graphs (REF13:918-921); the reverse sums the replicas
def _repeat_fwd(consts, img: Tensor):
    return [K.repeat_graphs(img.contiguous(), consts[0])], []


def _repeat_bwd(consts, inputs, outs, saved, gouts, needs):
    g = gouts[0]
    b, c, h, w = g.shape
    return (g.reshape(b, consts[0], c // consts[0], h, w).sum(1),)


def _repeat_fake(consts, img: Tensor):
    b, c, h, w = img.shape
    return [_new(img, b, consts[0] * c, h, w)], []


REPEAT_GRAPHS = OpaqueFunction("repeat_graphs_train", 1, _repeat_fwd, _repeat_bwd, _repeat_fake)


class Conv1x1Fn:
    @staticmethod
    def apply(x: Tensor, weight: Tensor) -> Tensor:
        return CONV1X1([], x, weight)


class Conv2x2s2Fn:
    @staticmethod
    def apply(x: Tensor, weight: Tensor) -> Tensor:
        return CONV2X2S2([], x, weight)


class RepeatGraphsFn:
    @staticmethod
    def apply(img: Tensor, n_graphs: int) -> Tensor:
        return REPEAT_GRAPHS([n_graphs], img)


# ---- GLRFast / GTVFast / extract_edge_weights sub-API (REF:146-237, :391-523) ----------
def _taps_params(module) -> Tuple[Tensor, ...]:
    return (module.stats_kernel_p01, module.stats_kernel_p02a, module.stats_kernel_p02b, module.stats_kernel_p03)


GLR_KIND, GTV_KIND = 0, 1


# GLRFast.forward (GLR_KIND: S^T (I - W) S x) or GTVFast.forward (GTV_KIND: C^T C x)
def _graph_apply_fwd(consts, x: Tensor, w: Tensor, p01, p02a, p02b, p03):
    kind, g = consts
    st = Stencil(*[t.data_ptr() for t in (p01, p02a, p02b, p03)])
    if kind == GLR_KIND:
        return [K.system_half(x, w, None, st, K.NO_STENCIL, None, None, g)], []
    c = K.gtv_pair_weights(w)
    return [K.system_half(x, None, c, K.NO_STENCIL, st, None, None, g)], [c]


def _graph_apply_bwd(consts, inputs, outs, saved, gouts, needs):
    kind, g = consts
    x, w, p01, p02a, p02b, p03 = inputs
    gout = gouts[0].contiguous()
    taps = K.stencil_taps(p01, p02a, p02b, p03)
    one = torch.ones(g, dtype=torch.float32, device=x.device)
    gx, gw, gtaps = torch.zeros_like(x), torch.zeros_like(w), torch.zeros_like(taps)
    if kind == GLR_KIND:
        glr_term_bwd(x, gout, taps, w, one, 1.0, g, gx, gw, None, gtaps)
    else:
        c = saved[0]
        gc = torch.zeros_like(c)
        gtv_term_bwd(x, gout, taps, c, one, 1.0, g, gx, gc, None, gtaps)
        K.bwd_pair_weights(w, gc, gw)
    return (gx, gw, *K.stencil_taps_backward(gtaps))


def _graph_apply_fake(consts, x: Tensor, w: Tensor, *taps):
    b, g, _, h, ww = w.shape
    return [torch.empty_like(x)], ([] if consts[0] == GLR_KIND else [_new(w, b, g, 2, h, ww)])


GRAPH_APPLY = OpaqueFunction("graph_apply_train", 1, _graph_apply_fwd, _graph_apply_bwd, _graph_apply_fake)


def graph_apply(module, kind: str, x5: Tensor, w: Tensor) -> Tensor:
    b, g, f, h, ww = x5.shape
    out = GRAPH_APPLY([GLR_KIND if kind == "glr" else GTV_KIND, g], x5.reshape(b, g * f, h, ww).contiguous(),
                      w.contiguous(), *_taps_params(module))
    return out.view(b, g, f, h, ww)


# extract_edge_weights: features [B,G*F,H,W] -> (w [B,G,4,H,W], degree [B,G,H,W])
def _edge_weights_fwd(consts, feat: Tensor, multiM: Tensor):
    g = consts[0]
    w, deg = K.edge_weights(feat, 0, g, feat.shape[1] // g, multiM, with_degree=True)
    return [w, deg], []


def _edge_weights_bwd(consts, inputs, outs, saved, gouts, needs):
    feat, multiM = inputs
    w = outs[0]
    gw, gdeg = gouts
    g = consts[0]
    gw_t = torch.zeros_like(w) if gw is None else gw.contiguous().clone()
    if gdeg is not None:                      # degree = sum_e w_e
        gw_t += gdeg.unsqueeze(2)
    gfeat, gM = torch.empty_like(feat), torch.zeros_like(multiM)
    K.bwd_edge_weights(feat, 0, g, feat.shape[1] // g, multiM, w, gw_t, gfeat, gM)
    return gfeat, gM


def _edge_weights_fake(consts, feat: Tensor, multiM: Tensor):
    b, _, h, w = feat.shape
    g = consts[0]
    return [_new(feat, b, g, 4, h, w), _new(feat, b, g, h, w)], []


EDGE_WEIGHTS = OpaqueFunction("edge_weights_train", 2, _edge_weights_fwd, _edge_weights_bwd, _edge_weights_fake)


def edge_weights(module, f5: Tensor):
    b, g, f, h, w = f5.shape
    return EDGE_WEIGHTS([g], f5.reshape(b, g * f, h, w).contiguous(), module.multiM)


# ---- v10 MixtureGLR (lib/model_GLR_GTV_deep_v10.py:241-335) -----------------------------
V10_PARAMS = ("GLRmodule00.multiM",) + tuple(f"GLRmodule00.{q}" for q in STENCIL_PARAMS) + (
    "muys00", "alphaCGD", "betaCGD")


# (y, feat, params) -> x_S of the GLR-only heavy-ball solver, A = I + mu L with mu linear
def _glr_fwd(consts, y: Tensor, feat: Tensor, *params: Tensor):
    p = dict(zip(V10_PARAMS, params))
    g = consts[0]
    wL, _ = K.edge_weights(feat, 0, g, y.shape[1] // g, p["GLRmodule00.multiM"])
    st = Stencil(*[p[f"GLRmodule00.{q}"].data_ptr() for q in STENCIL_PARAMS])
    mu, alpha, beta = p["muys00"], p["alphaCGD"], p["betaCGD"]
    n_st = alpha.shape[0]
    x, u = K.glr_stage(y, y, None, wL, st, mu, alpha[0], None, g)       # u_0 = r_0, x_1
    xs, us = [y, x], [u]
    for k in range(1, n_st):
        x, u = K.glr_stage(x, y, u, wL, st, mu, alpha[k], beta[k], g)
        xs.append(x)
        us.append(u)
    return [xs[-1]], [wL, *xs[1:-1], *us]


def _glr_fake(consts, y: Tensor, feat: Tensor, *params: Tensor):
    b, c, h, w = y.shape
    n_st = dict(zip(V10_PARAMS, params))["alphaCGD"].shape[0]
    return [torch.empty_like(y)], [_new(y, b, consts[0], 4, h, w), *[torch.empty_like(y) for _ in range(2 * n_st - 1)]]


def _glr_bwd(consts, inputs, outs, saved, gouts, needs):
    g = consts[0]
    y, feat = inputs[:2]
    params = inputs[2:]
    n_st = len(saved) // 2
    wL = saved[0]
    xs = (y,) + tuple(saved[1:n_st])        # x_0 = y, x_1 .. x_{S-1}
    us = saved[n_st:]                       # u_0 .. u_{S-1}
    p = dict(zip(V10_PARAMS, params))
    mu, alpha, beta = p["muys00"], p["alphaCGD"], p["betaCGD"]
    taps = K.stencil_taps(*[p[f"GLRmodule00.{q}"] for q in STENCIL_PARAMS])
    gw, gtaps, gmu = torch.zeros_like(wL), torch.zeros_like(taps), torch.zeros_like(mu)
    galpha, gbeta = torch.zeros_like(alpha), torch.zeros_like(beta)
    gy = torch.zeros_like(y)
    gx = gouts[0].contiguous()
    gu_next = None
    for k in range(n_st - 1, -1, -1):
        # x_{k+1} = x_k + a_k u_k,  u_k = (y - A x_k) + b_k u_{k-1}   (u_{-1} = 0; x_0 = y)
        gu, gx = cg_glue(gx, us[k], gu_next, us[k - 1] if k >= 1 else None, alpha, beta, gy, galpha, gbeta,
                         k, g, owned=k < n_st - 1)                     # gx <- gx_{k+1} - gu
        if k >= 1:
            glr_term_bwd(xs[k], gu, taps, wL, mu, -1.0, g, gx, gw, gmu, gtaps)
        else:                                                           # x_0 = y
            gy.add_(gx)
            glr_term_bwd(y, gu, taps, wL, mu, -1.0, g, gy, gw, gmu, gtaps)
        gu_next = gu
    gfeat, gM = torch.empty_like(feat), torch.zeros_like(p["GLRmodule00.multiM"])
    K.bwd_edge_weights(feat, 0, g, y.shape[1] // g, p["GLRmodule00.multiM"], wL, gw, gfeat, gM)
    grads = {"GLRmodule00.multiM": gM, "muys00": gmu, "alphaCGD": galpha, "betaCGD": gbeta}
    for q, gq in zip(STENCIL_PARAMS, K.stencil_taps_backward(gtaps)):
        grads[f"GLRmodule00.{q}"] = gq
    return (gy, gfeat, *[grads[n] for n in V10_PARAMS])


GLR_SOLVE = OpaqueFunction("glr_solve_train", 1, _glr_fwd, _glr_bwd, _glr_fake)


def glr_solve(mod, y: Tensor, feat: Tensor) -> Tensor:
    params = [mod.GLRmodule00.multiM] + [getattr(mod.GLRmodule00, q) for q in STENCIL_PARAMS] + [
        mod.muys00, mod.alphaCGD, mod.betaCGD]
    return GLR_SOLVE([mod.n_graphs], y, feat.contiguous(), *params)


# ---- two-scale GLR-only solver (config C2; glr_v10.MultiScaleMixtureGLR) ---------------------
GLR2_PARAMS = ("GLRmodule00.multiM", "GLRmodule01.multiM") + tuple(
    f"{m}.{q}" for m in ("GLRmodule00", "GLRmodule01") for q in STENCIL_PARAMS) + (
    "muys00", "muys01", "alphaCGD", "betaCGD")


# (y, f0, f1, params) -> x_S of  A = I + e^mu0 L0 + U e^mu1 L1 D  under the v10 recurrence
def _glr2_fwd(consts, y: Tensor, f0: Tensor, f1: Tensor, *params: Tensor):
    p = dict(zip(GLR2_PARAMS, params))
    g = consts[0]
    nf = y.shape[1] // g
    wL0, _ = K.edge_weights(f0, 0, g, nf, p["GLRmodule00.multiM"])
    wL1, _ = K.edge_weights(f1, 0, g, nf, p["GLRmodule01.multiM"])
    sL0 = Stencil(*[p[f"GLRmodule00.{q}"].data_ptr() for q in STENCIL_PARAMS])
    sL1 = Stencil(*[p[f"GLRmodule01.{q}"].data_ptr() for q in STENCIL_PARAMS])
    mu0, mu1, alpha, beta = p["muys00"], p["muys01"], p["alphaCGD"], p["betaCGD"]
    n_st = alpha.shape[0]
    x, u, xd = y, None, K.pool2(y)
    xs, us = [y], []
    for k in range(n_st):
        t = K.system_half(xd, wL1, None, sL1, K.NO_STENCIL, mu1, None, g)
        x, u, xd = K.system_step(x, y, u, t, wL0, None, sL0, K.NO_STENCIL, mu0, None, alpha[k],
                                 beta[k] if k >= 1 else None, g, want_u=True, want_pool=k < n_st - 1)
        xs.append(x)
        us.append(u)
    return [xs[-1]], [wL0, wL1, *xs[1:-1], *us]


def _glr2_fake(consts, y: Tensor, f0: Tensor, f1: Tensor, *params: Tensor):
    b, c, h, w = y.shape
    g = consts[0]
    n_st = dict(zip(GLR2_PARAMS, params))["alphaCGD"].shape[0]
    return [torch.empty_like(y)], [_new(y, b, g, 4, h, w), _new(y, b, g, 4, h // 2, w // 2),
                                   *[torch.empty_like(y) for _ in range(2 * n_st - 1)]]


def _glr2_bwd(consts, inputs, outs, saved, gouts, needs):
    g = consts[0]
    y, f0, f1 = inputs[:3]
    params = inputs[3:]
    n_st = (len(saved) - 1) // 2
    wL0, wL1 = saved[:2]
    xs = (y,) + tuple(saved[2:2 + n_st - 1])      # x_0 = y, x_1 .. x_{S-1}
    us = saved[2 + n_st - 1:]                     # u_0 .. u_{S-1}
    p = dict(zip(GLR2_PARAMS, params))
    mu0, mu1 = torch.exp(p["muys00"]), torch.exp(p["muys01"])
    alpha, beta = p["alphaCGD"], p["betaCGD"]
    taps0 = K.stencil_taps(*[p[f"GLRmodule00.{q}"] for q in STENCIL_PARAMS])
    taps1 = K.stencil_taps(*[p[f"GLRmodule01.{q}"] for q in STENCIL_PARAMS])
    gw0, gw1 = torch.zeros_like(wL0), torch.zeros_like(wL1)
    gt0, gt1 = torch.zeros_like(taps0), torch.zeros_like(taps1)
    gm0, gm1 = torch.zeros_like(mu0), torch.zeros_like(mu1)
    galpha, gbeta = torch.zeros_like(alpha), torch.zeros_like(beta)
    gy = torch.zeros_like(y)

    def a_bwd(x: Tensor, gu: Tensor, out: Tensor) -> None:     # out -= (A - I)^T gu (+ params)
        glr_term_bwd(x, gu, taps0, wL0, mu0, -1.0, g, out, gw0, gm0, gt0)
        xd, gd = K.pool2(x), K.pool2(gu)                       # U^T = D
        gxd = torch.zeros_like(xd)
        glr_term_bwd(xd, gd, taps1, wL1, mu1, -1.0, g, gxd, gw1, gm1, gt1)
        K.bwd_unpool2_acc(gxd, out)                            # D^T = U

    gx = gouts[0].contiguous()
    gu_next = None
    for k in range(n_st - 1, -1, -1):
        gu, gx = cg_glue(gx, us[k], gu_next, us[k - 1] if k >= 1 else None, alpha, beta, gy, galpha, gbeta,
                         k, g, owned=k < n_st - 1)                     # gx <- gx_{k+1} - gu
        if k >= 1:
            a_bwd(xs[k], gu, gx)
        else:                                                           # x_0 = y
            gy.add_(gx)
            a_bwd(y, gu, gy)
        gu_next = gu
    nf = y.shape[1] // g
    gf0, gf1 = torch.empty_like(f0), torch.empty_like(f1)
    gM0, gM1 = torch.zeros_like(p["GLRmodule00.multiM"]), torch.zeros_like(p["GLRmodule01.multiM"])
    K.bwd_edge_weights(f0, 0, g, nf, p["GLRmodule00.multiM"], wL0, gw0, gf0, gM0)
    K.bwd_edge_weights(f1, 0, g, nf, p["GLRmodule01.multiM"], wL1, gw1, gf1, gM1)
    grads = {"GLRmodule00.multiM": gM0, "GLRmodule01.multiM": gM1, "muys00": gm0 * mu0, "muys01": gm1 * mu1,
             "alphaCGD": galpha, "betaCGD": gbeta}
    for m, gt in (("GLRmodule00", gt0), ("GLRmodule01", gt1)):
        for q, gq in zip(STENCIL_PARAMS, K.stencil_taps_backward(gt)):
            grads[f"{m}.{q}"] = gq
    return (gy, gf0, gf1, *[grads[n] for n in GLR2_PARAMS])


GLR2_SOLVE = OpaqueFunction("glr2_solve_train", 1, _glr2_fwd, _glr2_bwd, _glr2_fake)


def glr2_solve(mod, y: Tensor, f0: Tensor, f1: Tensor) -> Tensor:
    params = []
    for name in GLR2_PARAMS:
        obj = mod
        for part in name.split("."):
            obj = getattr(obj, part)
        params.append(obj)
    return GLR2_SOLVE([mod.n_graphs], y, f0.contiguous(), f1.contiguous(), *params)


# ---- LocalNonLinearBlock (nsubnets = 1; REF:911-964, REF13:541-575) ---------------------
def _mat(w: Tensor, rows: int) -> Tensor:
    return w.reshape(rows, -1)


# out = s0 x + s1 W2 gate(dw3x3(W1 LN(x))): fused HIP forward; the reverse recomputes n, h, h', gate
# with HIP kernels and runs the adjoints (GEMMs: HIP conv1x1 for the data gradients, one library GEMM
# per weight gradient)
# The eager forward keeps the head's gated activation g (a view of the launch's workspace) for the
# reverse's W2 weight gradient, which then skips recomputing the depthwise + gate.  g costs hid floats
# per pixel, so the gates alive at once are capped by a budget derived from the device's memory
# (KEEP_GATE_FRACTION of it: 32 GB of a 288 GB MI355X -- all of the msgf step's gates, about three
# quarters of the C4 shape's C <= 128 blocks, whose step already holds ~142 GB -- and proportionally
# less on a smaller device; KEEP_GATE_BYTES, when set, overrides it); a kept gate leaves the budget when
# its tensor is freed.  Compiled graphs always recompute (the custom op's saved list is fixed).
KEEP_GATE = True
KEEP_GATE_FRACTION = 1.0 / 9.0
KEEP_GATE_BYTES = None
_KEPT = [0]
_GATE_BUDGET = {}


def keep_gate_budget(device) -> int:
    """Bytes of kept gates allowed alive at once on ``device``."""
    if KEEP_GATE_BYTES is not None:
        return int(KEEP_GATE_BYTES)
    idx = torch.device(device).index or 0
    if idx not in _GATE_BUDGET:
        _GATE_BUDGET[idx] = int(KEEP_GATE_FRACTION * torch.cuda.get_device_properties(idx).total_memory)
    return _GATE_BUDGET[idx]


def _unkeep(nbytes: int) -> None:
    _KEPT[0] -= nbytes


def _lnb_keeps_gate(x: Tensor, w2: Tensor) -> bool:
    b, c, h, w = x.shape
    return KEEP_GATE and FUSED_GATE_DW3 and K.lnb_gate_dw3_ok(h, w) and K.lnb_gate_keepable(c, w2.shape[1], h, w)


def _lnb_fwd(consts, x: Tensor, ln_w: Tensor, w1: Tensor, wdw: Tensor, w2: Tensor, skip: Tensor):
    c, hid2 = x.shape[1], w1.shape[0]
    args = (x.contiguous(), ln_w.reshape(c).contiguous(), _mat(w1, hid2).contiguous(), _mat(wdw, hid2).contiguous(),
            _mat(w2, c).contiguous(), skip.contiguous())
    if consts and consts[0] and _lnb_keeps_gate(x, w2):
        b, _, h, w = x.shape
        nbytes = 4 * b * w2.shape[1] * h * w
        if _KEPT[0] + nbytes <= keep_gate_budget(x.device):
            out, gate = K.lnb_forward_keep(*args)
            _KEPT[0] += nbytes
            weakref.finalize(gate, _unkeep, nbytes)
            return [out], [gate]
    return [K.lnb_forward(*args)], []


def _lnb_fake(consts, x: Tensor, *weights: Tensor):
    return [torch.empty_like(x)], []


def _lnb_bwd(consts, inputs, outs, saved, gouts, needs):
    x, ln_w, w1, wdw, w2, skip = inputs
    gout = gouts[0].contiguous()
    b, c, h, w = x.shape
    hid2 = w1.shape[0]
    hid = hid2 // 2
    lnw, W1, Wdw, W2 = ln_w.reshape(c).contiguous(), _mat(w1, hid2).contiguous(), _mat(wdw, hid2).contiguous(), \
        _mat(w2, c).contiguous()
    n, isd = K.lnb_norm(x, lnw)
    hh = K.conv1x1(n, W1.view(hid2, c, 1, 1))
    # row-kernel widths: the depthwise output hp is never stored (gate from hh in one pass, the
    # reverse recomputes hp from hh); else the per-stage kernels
    rows = FUSED_GATE_DW3 and K.lnb_gate_dw3_ok(h, w)
    if rows:
        hp = None
        gate = saved[0] if saved else K.lnb_dw3_gate(hh, Wdw)
    else:
        hp = K.dwconv3(hh, Wdw)
        gate, _ = K.lnb_gate(hp)
    gskip = torch.zeros(2, dtype=torch.float32, device=x.device)
    if not LN_SKIP_FUSED:
        K.bwd_graph_dot(gout, x, gskip[0:1], 1)
    s1 = skip[1:2].contiguous()
    # gw2 = s1 gout gate^T; gq = W2^T gout: the gate reverse takes s1 and returns
    # <gout, W2 gate> = <gq, gate> for the skip weight (no recomputed W2 gate)
    gw2 = K.wgrad(gout.contiguous(), gate.contiguous()) * s1
    del gate
    gq = K.conv1x1(gout, W2.t().contiguous().view(hid, c, 1, 1))
    gwdw = torch.zeros_like(Wdw)
    if rows:                                        # ghp formed in registers, never in HBM
        gh = K.lnb_gate_dw3_bwd(None, gq, s1, hh, Wdw, gwdw, gskip[1:2])
        del hp, gq, hh
    else:
        ghp = K.lnb_gate_bwd_scaled(hp, gq, s1, gskip[1:2])
        del hp, gq
        gh = K.dwconv3_bwd(ghp, hh, Wdw, gwdw)
        del ghp, hh
    gw1 = K.wgrad(gh.contiguous(), n.contiguous())
    gn = K.conv1x1(gh, W1.t().contiguous().view(c, hid2, 1, 1))
    del gh, n
    gx, glnw = _ln_skip_bwd(x, lnw, isd, gn, gout, skip, gskip)
    return gx, glnw.view_as(ln_w), gw1.view_as(w1), gwdw.view_as(wdw), gw2.view_as(w2), gskip


def _ln_skip_bwd(x: Tensor, lnw: Tensor, isd: Tensor, gn: Tensor, gout: Tensor, skip: Tensor, gskip: Tensor):
    """gx = s0 gout + the norm's data gradient, gskip[0] += <gout, x> (the skip weight), and the norm's
    weight gradient: one pass over gout (grr_lnb_norm_bwd_skip) or the dot / scale / norm passes."""
    glnw = torch.zeros_like(lnw)
    if LN_SKIP_FUSED:
        return K.lnb_norm_bwd_skip(x, lnw, isd, gn, gout, skip.contiguous(), glnw, gskip[0:1]), glnw
    gx = K.bwd_lincomb(gout, skip[0:1].contiguous(), None, None, 1)          # s0 * gout
    K.lnb_norm_bwd(x, lnw, isd, gn, gx, glnw)
    return gx, glnw


LNB = OpaqueFunction("lnb_train", 1, _lnb_fwd, _lnb_bwd, _lnb_fake)


class LNBFn:
    @staticmethod
    def apply(x: Tensor, ln_w: Tensor, w1: Tensor, wdw: Tensor, w2: Tensor, skip: Tensor) -> Tensor:
        # consts [1]: the eager forward may keep the gate (a compiled graph's saved list must not vary)
        eager = not (train_ops.FORCE_OPS or torch.compiler.is_compiling())
        return LNB([1 if eager else 0], x, ln_w, w1, wdw, w2, skip)


# ---- FFBlock of the window models' feature CNN (REF7:13-67), training --------------------------
# out = s0 x + s1 W_out (gelu(d1) d2), [d1; d2] = dwconv3x3_zero(W_in LN(x)): HIP forward
# (grr_ffn_forward); the reverse recomputes n, hh and the gate and runs the adjoints on HIP kernels
# (split-bf16 GEMMs for the data gradients, grr_wgrad for the weight gradients, one row pass for the
# gate + depthwise reverse).  Row kernels: W <= 256 (the window models train on 64 / 256 patches).
def _ffn_fwd(consts, x: Tensor, ln_w: Tensor, w_in: Tensor, w_dw: Tensor, w_out: Tensor, skip: Tensor):
    c, hid2 = x.shape[1], w_in.shape[0]
    out = K.ffn_forward(x.contiguous(), ln_w.reshape(c).contiguous(), _mat(w_in, hid2).contiguous(),
                        _mat(w_dw, hid2).contiguous(), _mat(w_out, c).contiguous(), skip.contiguous())
    return [out], []


def _ffn_bwd(consts, inputs, outs, saved, gouts, needs):
    x, ln_w, w_in, w_dw, w_out, skip = inputs
    gout = gouts[0].contiguous()
    b, c, h, w = x.shape
    hid2 = w_in.shape[0]
    hid = hid2 // 2
    lnw, Win, Wdw, Wout = ln_w.reshape(c).contiguous(), _mat(w_in, hid2).contiguous(), \
        _mat(w_dw, hid2).contiguous(), _mat(w_out, c).contiguous()
    n, isd = K.lnb_norm(x, lnw)
    hh = K.conv1x1(n, Win.view(hid2, c, 1, 1))
    gate = K.ffn_dw3_gate(hh, Wdw)
    gskip = torch.zeros(2, dtype=torch.float32, device=x.device)
    if not LN_SKIP_FUSED:
        K.bwd_graph_dot(gout, x, gskip[0:1], 1)
    s1 = skip[1:2].contiguous()
    gw_out = K.wgrad(gout, gate) * s1                  # d/dW_out of s1 W_out gate
    del gate
    gq = K.conv1x1(gout, Wout.t().contiguous().view(hid, c, 1, 1))
    gwdw = torch.zeros_like(Wdw)
    gh = K.ffn_gate_dw3_bwd(gq, s1, hh, Wdw, gwdw, gskip[1:2])   # <gq, gate> = <gout, W_out gate>
    del gq, hh
    gw_in = K.wgrad(gh, n)
    gn = K.conv1x1(gh, Win.t().contiguous().view(c, hid2, 1, 1))
    del gh, n
    gx, glnw = _ln_skip_bwd(x, lnw, isd, gn, gout, skip, gskip)
    return gx, glnw.view_as(ln_w), gw_in.view_as(w_in), gwdw.view_as(w_dw), gw_out.view_as(w_out), gskip


FFN = OpaqueFunction("ffn_train", 1, _ffn_fwd, _ffn_bwd, _lnb_fake)


class FFNFn:
    @staticmethod
    def apply(x: Tensor, ln_w: Tensor, w_in: Tensor, w_dw: Tensor, w_out: Tensor, skip: Tensor) -> Tensor:
        return FFN([], x, ln_w, w_in, w_dw, w_out, skip)


# ---- the GLRFast / GTVFast module methods, differentiable (REF:128-228, :452-516) ------------
# Forward: the standalone sub-API kernels (csrc/subapi_ops.hip); reverse: csrc/subapi_bwd.hip.
# Stencil inputs are the module's four stats_kernel_p* parameters; tap gradients come back per
# channel [G*F, 5] and are chained to them by kernels.stencil_taps_backward.
def _st4(ps) -> Stencil:
    return Stencil(*[p.data_ptr() for p in ps])


def _neighbors_fwd(consts, x: Tensor):
    return [K.neighbor_gather(x.contiguous())], []


def _neighbors_bwd(consts, inputs, outs, saved, gouts, needs):
    return (K.neighbor_gather_bwd(gouts[0].contiguous()),)


def _neighbors_fake(consts, x: Tensor):
    b, c, h, w = x.shape
    return [_new(x, b, c, 4, h, w)], []


NEIGHBORS = OpaqueFunction("neighbor_gather_train", 1, _neighbors_fwd, _neighbors_bwd, _neighbors_fake)


def _normalize_fwd(consts, f5: Tensor, multiM: Tensor):
    return [K.normalize_features(f5.contiguous(), multiM.contiguous())], []


def _normalize_bwd(consts, inputs, outs, saved, gouts, needs):
    f5, multiM = inputs
    b, g, f, h, w = f5.shape
    gM = torch.zeros_like(multiM)
    gf = K.normalize_features_bwd(f5.contiguous(), multiM.contiguous(), gouts[0].contiguous().view(b, g, f, h, w), gM)
    return gf, gM


def _normalize_fake(consts, f5: Tensor, multiM: Tensor):
    b, g, f, h, w = f5.shape
    return [_new(f5, b, g * f, h, w)], []


NORMALIZE = OpaqueFunction("normalize_features_train", 1, _normalize_fwd, _normalize_bwd, _normalize_fake)


def _taps_grads(gtaps: Tensor, ps) -> Tuple[Tensor, ...]:
    return tuple(gq.view_as(p) for gq, p in zip(K.stencil_taps_backward(gtaps), ps))


def _stats_fwd(consts, x5: Tensor, *ps: Tensor):
    return [K.stats_conv(x5.contiguous(), _st4(ps), bool(consts[0]))], []


def _stats_bwd(consts, inputs, outs, saved, gouts, needs):
    x5, ps = inputs[0], inputs[1:]
    gtaps = torch.zeros((x5.shape[1] * x5.shape[2], 5), dtype=torch.float32, device=x5.device)
    gx = K.stats_conv_bwd(x5.contiguous(), _st4(ps), bool(consts[0]), gouts[0].contiguous(), gtaps)
    return (gx, *_taps_grads(gtaps, ps))


def _stats_fake(consts, x5: Tensor, *ps: Tensor):
    return [torch.empty_like(x5)], []


STATS_CONV = OpaqueFunction("stats_conv_train", 1, _stats_fwd, _stats_bwd, _stats_fake)


def _lnorm_fwd(consts, x5: Tensor, w: Tensor):
    return [K.glr_op_L_norm(x5.contiguous(), w.contiguous())], []


def _lnorm_bwd(consts, inputs, outs, saved, gouts, needs):
    x5, w = inputs
    return K.glr_op_L_norm_bwd(x5.contiguous(), w.contiguous(), gouts[0].contiguous())


def _lnorm_fake(consts, x5: Tensor, w: Tensor):
    return [torch.empty_like(x5)], []


OP_L_NORM = OpaqueFunction("glr_op_L_norm_train", 1, _lnorm_fwd, _lnorm_bwd, _lnorm_fake)


def _opc_fwd(consts, x5: Tensor, w: Tensor, *ps: Tensor):
    return [K.gtv_op_C(x5.contiguous(), w.contiguous(), _st4(ps))], []


def _opc_bwd(consts, inputs, outs, saved, gouts, needs):
    x5, w, ps = inputs[0], inputs[1], inputs[2:]
    gtaps = torch.zeros((x5.shape[1] * x5.shape[2], 5), dtype=torch.float32, device=x5.device)
    gx, gw = K.gtv_op_C_bwd(x5.contiguous(), w.contiguous(), _st4(ps), gouts[0].contiguous(), gtaps)
    return (gx, gw, *_taps_grads(gtaps, ps))


def _opc_fake(consts, x5: Tensor, w: Tensor, *ps: Tensor):
    b, g, f, h, ww = x5.shape
    return [_new(x5, b, g, f, 4, h, ww)], []


OP_C = OpaqueFunction("gtv_op_C_train", 1, _opc_fwd, _opc_bwd, _opc_fake)


def _opct_fwd(consts, e6: Tensor, w: Tensor, *ps: Tensor):
    out, z = K.gtv_op_C_transpose(e6.contiguous(), w.contiguous(), _st4(ps), want_work=True)
    return [out], [z]


def _opct_bwd(consts, inputs, outs, saved, gouts, needs):
    e6, w, ps = inputs[0], inputs[1], inputs[2:]
    gtaps = torch.zeros((e6.shape[1] * e6.shape[2], 5), dtype=torch.float32, device=e6.device)
    gE, gw = K.gtv_op_C_transpose_bwd(e6.contiguous(), w.contiguous(), _st4(ps), saved[0], gouts[0].contiguous(),
                                      gtaps)
    return (gE, gw, *_taps_grads(gtaps, ps))


def _opct_fake(consts, e6: Tensor, w: Tensor, *ps: Tensor):
    b, g, f, _, h, ww = e6.shape
    return [_new(e6, b, g, f, h, ww)], [_new(e6, b, g, f, h, ww)]


OP_C_T = OpaqueFunction("gtv_op_C_transpose_train", 1, _opct_fwd, _opct_bwd, _opct_fake)
