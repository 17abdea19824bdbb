"""Reverse pass of the window-graph MixtureGTV solver (REF7 / REF1) on the HIP kernels.

REF7 = exploration/model_multiscale_mixture_GLR/lib/model_GLR_GTV_deep_v7.py
(MixtureGTV :802-1016), REF1 = lib/model_GLR_GTV_deep_v1.py (:472-676, identity stats
stencil).  The reference trains these models through PyTorch autograd over materialised
[B,G,Fs,K,H,W] edge tensors (the multiblocks training script).  Here the forward runs the
fused inference kernels of window_ops.hip, keeping the iterates the reverse needs, and the
reverse sweep is written out on the adjoint kernels of window_bwd.hip:

  group A   x_0 = r_0 = y + ro G y;  2 stages                          (REF7:945-958)
  prox rhs  r_1 = y + ro S^T C^T phi(C S x_2)                           (REF7:958-967)
  group B   x = r_1;  stages 2 .. S-1                                    (REF7:970-990)
  stage     x' = x + a_k u_k,  u_k = (r - A x) + b_k u_{k-1}  (no b in a group's first stage)
            -> ga_k = <gx', u_k>_g, gu_k = a_k gx' + b_{k+1} gu_{k+1}, gb_k = <gu_k, u_{k-1}>_g,
               gx = gx' - A^T gu_k, gr += gu_k (and gr += gx at a group's first stage)
  operator  A = I + mu S_L^T (I - W_L) S_L + ro S_G^T C^T C S_G,  mu / ro linear, gamma = exp
  weights   softmax over K similarities of normalised, multiM-scaled features (REF7:418-446)
  mixture   out = sum_g softmax(conv1x1(features))_g x_g + dc                  (REF7:1006-1009)

The bare module calls differentiate the same way: ``WinEdgeWeightsFn`` is
``GLRFast/GTVFast.extract_edge_weights`` (REF7:418-446, REF1:255-272) and ``WinOperatorFn`` their
``forward`` (REF7:503-511 / :776-782, REF1:274-291 / :421-470), each with its HIP reverse.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch

from . import kernels as K

Tensor = torch.Tensor

STENCIL_PARAMS = ("stats_kernel_p01", "stats_kernel_p02a", "stats_kernel_p02b", "stats_kernel_p03")
BASE_PARAMS = ("GTVmodule00.multiM", "GLRmodule00.multiM", "ro00", "gamma00", "muys00", "alphaCGD", "betaCGD")
TAP_PARAMS = tuple(f"{m}.{q}" for m in ("GTVmodule00", "GLRmodule00") for q in STENCIL_PARAMS)


def param_names(with_taps: bool) -> Tuple[str, ...]:
    return BASE_PARAMS + (TAP_PARAMS if with_taps else ())


def _get(mod, name: str) -> Tensor:
    obj = mod
    for part in name.split("."):
        obj = getattr(obj, part)
    return obj


def taps_backward(gt: Tensor) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """Chain rule of K.win_taps: taps = (p01 - p02a - p02b + 4 p03, -p03, -p03, p02a - p03, p02b - p03)."""
    c, u, l, r, d = gt.unbind(0)
    return ((c).reshape(1), (r - c).reshape(1), (d - c).reshape(1), (4 * c - u - l - r - d).reshape(1))


class _Terms:
    """The operator's two graphs: weights, stencils, scalars and their gradient buffers."""

    def __init__(self, wG, wL, tG, tL, ro, mu, log_gamma, delta, g):
        self.wG, self.wL, self.tG, self.tL = wG, wL, tG, tL
        self.ro, self.mu, self.log_gamma = ro, mu, log_gamma
        self.delta, self.g = delta, g
        z = torch.zeros_like
        self.gwG, self.gwL = z(wG), z(wL)
        self.gtG, self.gtL = z(tG), z(tL)
        self.gro, self.gmu, self.ggam = z(ro), z(mu), z(log_gamma)

    def glr_bwd(self, x: Tensor, gg: Tensor, coef: float, out: Tensor) -> None:
        """out += coef mu P*(I-W)^T T* gg; gradients of <coef gg, mu T (I-W) P x>."""
        g = self.g
        sc = self.mu * coef
        s = K.win_bwd_stencil(x, self.tL, K.WST_P, g)
        bt = K.win_bwd_stencil(gg, self.tL, K.WST_T_ADJ, g)
        l, gs = K.win_bwd_glr(s, bt, self.wL, self.delta, sc, coef, self.gwL, self.gmu, g)
        del s, bt
        K.win_bwd_tapgrad(gg, l, K.WTAP_T, g, sc, self.gtL)
        K.win_bwd_tapgrad(gs, x, K.WTAP_P, g, None, self.gtL)
        K.win_bwd_stencil(gs, self.tL, K.WST_P_ADJ, g, None, out=out)

    def gtv_bwd(self, x: Tensor, gg: Tensor, coef: float, out: Tensor, prox: bool = False) -> None:
        """out += coef ro P* C^T-reverse T* gg (prox: C^T phi(C .)); parameter gradients."""
        g = self.g
        sc = self.ro * coef
        s = K.win_bwd_stencil(x, self.tG, K.WST_P, g)
        bt = K.win_bwd_stencil(gg, self.tG, K.WST_T_ADJ, g)
        o, gs = K.win_bwd_gtv(s, bt, self.wG, self.delta, prox, self.log_gamma if prox else None, sc, coef,
                              self.gwG, self.gro, self.ggam if prox else None, g)
        del s, bt
        K.win_bwd_tapgrad(gg, o, K.WTAP_T, g, sc, self.gtG)
        K.win_bwd_tapgrad(gs, x, K.WTAP_P, g, None, self.gtG)
        K.win_bwd_stencil(gs, self.tG, K.WST_P_ADJ, g, None, out=out)

    def a_bwd(self, x: Tensor, gg: Tensor, coef: float, out: Tensor) -> None:
        """out += coef (A - I)^T gg."""
        self.glr_bwd(x, gg, coef, out)
        self.gtv_bwd(x, gg, coef, out)


class _WindowSolve(torch.autograd.Function):
    """(y [B,Fs,H,W], feat [B,Ctot,H,W], params) -> x_S [B,G,Fs,H,W] of MixtureGTV's solver
    (REF7:936-1004), the graph features being channels [0, G*F) of feat."""

    @staticmethod
    def forward(ctx, spec, y: Tensor, feat: Tensor, *params: Tensor) -> Tensor:
        g, f, delta, with_taps = spec
        p = dict(zip(param_names(with_taps), params))
        fs = y.shape[1]
        wG, _ = K.win_edge_weights(feat, 0, g, f, p["GTVmodule00.multiM"].contiguous(), delta)
        wL, _ = K.win_edge_weights(feat, 0, g, f, p["GLRmodule00.multiM"].contiguous(), delta)
        if with_taps:
            tG = K.win_taps(*[p[f"GTVmodule00.{q}"] for q in STENCIL_PARAMS])
            tL = K.win_taps(*[p[f"GLRmodule00.{q}"] for q in STENCIL_PARAMS])
        else:
            tG = tL = torch.tensor(K.IDENTITY_TAPS, dtype=torch.float32, device=y.device)
        ro, mu, lg = p["ro00"].contiguous(), p["muys00"].contiguous(), p["gamma00"].contiguous()
        alpha, beta = p["alphaCGD"].contiguous(), p["betaCGD"].contiguous()
        n_st = alpha.shape[0]
        xs: List[Tensor] = []
        us: List[Tensor] = []
        # linear GTV passes on pair weights (as inference, window_graph.MixtureGTV.solve); the prox
        # rhs and the reverse use the raw directed weights
        from .window_graph import WIN_PAIR_WEIGHTS as pair
        cG = K.win_pair_weights(wG, delta) if pair else wG

        def stages(rhs, ks):
            x, u = rhs, None
            for k in ks:
                xs.append(x)
                x, u = K.win_solver(0, x, rhs, cG, tG, ro, delta, g, fs, wL=wL, tapsL=tL, mu=mu, alpha=alpha[k],
                                    beta=beta[k] if u is not None else None, u_prev=u, want_u=True, pair=pair)
                us.append(u)
            return x

        r0, _ = K.win_solver(1, y, y, cG, tG, ro, delta, g, fs, pair=pair)
        x2 = stages(r0, [0, 1])
        r1, _ = K.win_solver(2, x2, y, wG, tG, ro, delta, g, fs, log_gamma=lg)
        out = stages(r1, list(range(2, n_st)))
        del cG
        ctx.spec, ctx.n_st = spec, n_st
        ctx.save_for_backward(y, feat, wG, wL, tG, tL, x2, *params, *xs, *us)
        return out

    @staticmethod
    def backward(ctx, gout: Tensor):
        g, f, delta, with_taps = ctx.spec
        n_st = ctx.n_st
        names = param_names(with_taps)
        sv = ctx.saved_tensors
        y, feat, wG, wL, tG, tL, x2 = sv[:7]
        npar = len(names)
        params = sv[7:7 + npar]
        xs = sv[7 + npar:7 + npar + n_st]             # stage inputs: r0, x1, r1, x3, ..
        us = sv[7 + npar + n_st:]                      # u_0 .. u_{S-1}
        p = dict(zip(names, params))
        ro, mu, lg = p["ro00"].contiguous(), p["muys00"].contiguous(), p["gamma00"].contiguous()
        alpha, beta = p["alphaCGD"].contiguous(), p["betaCGD"].contiguous()
        T = _Terms(wG, wL, tG, tL, ro, mu, lg, delta, g)
        b, fs, h, w = y.shape
        galpha, gbeta = torch.zeros_like(alpha), torch.zeros_like(beta)

        def flat(t):                                   # [B,G,Fs,H,W] viewed as [B, G*Fs, H, W]
            return t.view(b, g * fs, h, w)

        gx = gout.contiguous()
        gy = torch.zeros_like(y)
        grhs = torch.zeros_like(gx)
        gu_next = None
        owned = False
        for k in range(n_st - 1, -1, -1):
            first = k in (0, 2)
            # ga_k, gu_k, gb_k, grhs += gu_k, gx' - gu_k in one pass (grr_bwd_cg_glue)
            gu, gxf = K.bwd_cg_glue(flat(gx), flat(us[k]), None if gu_next is None else flat(gu_next),
                                    None if first else flat(us[k - 1]), alpha[k],
                                    None if gu_next is None else beta[k + 1], flat(grhs), galpha[k],
                                    None if first else gbeta[k], g, inplace=owned)
            gu, gx, owned = gu.view_as(gx), gxf.view_as(gx), True
            T.a_bwd(xs[k], gu, -1.0, gx)                                           #   - (A - I)^T gu
            gu_next = gu
            if first:                                   # x_in = r: its gradient joins the rhs gradient
                grhs.add_(gx)
                if k == 2:                              # r1 = y + ro S^T C^T phi(C S x2)
                    gy.add_(grhs.sum(1))
                    gx = torch.zeros_like(grhs)
                    T.gtv_bwd(x2, grhs, 1.0, gx, prox=True)
                else:                                   # r0 = y + ro G y  (y shared by the graphs)
                    gy.add_(grhs.sum(1))
                    yr = y[:, None].expand(b, g, fs, h, w).contiguous()
                    gyr = torch.zeros_like(yr)
                    T.gtv_bwd(yr, grhs, 1.0, gyr)
                    gy.add_(gyr.sum(1))
                grhs = torch.zeros_like(grhs)
                gu_next = None
        del grhs, gu_next

        gfeat = torch.zeros_like(feat)
        gMG = torch.zeros_like(p["GTVmodule00.multiM"])
        gML = torch.zeros_like(p["GLRmodule00.multiM"])
        K.win_bwd_edge_weights(feat, 0, g, f, p["GTVmodule00.multiM"].contiguous(), wG, T.gwG, delta, gfeat, gMG)
        K.win_bwd_edge_weights(feat, 0, g, f, p["GLRmodule00.multiM"].contiguous(), wL, T.gwL, delta, gfeat, gML)
        grads = {"GTVmodule00.multiM": gMG, "GLRmodule00.multiM": gML, "ro00": T.gro,
                 "gamma00": T.ggam * torch.exp(lg), "muys00": T.gmu, "alphaCGD": galpha, "betaCGD": gbeta}
        if with_taps:
            for m, gt in (("GTVmodule00", T.gtG), ("GLRmodule00", T.gtL)):
                for q, gq in zip(STENCIL_PARAMS, taps_backward(gt)):
                    grads[f"{m}.{q}"] = gq.view_as(p[f"{m}.{q}"])
        return (None, gy, gfeat, *[grads[n] for n in names])


def window_solve(mod, y: Tensor, feat: Tensor, with_taps: bool) -> Tensor:
    """Differentiable MixtureGTV solve on the HIP kernels (graph features = channels [0, G*F) of feat)."""
    delta = tuple((int(a), int(c)) for a, c in mod.GTVmodule00.edge_delta)
    spec = (mod.n_graphs, mod.n_node_fts, delta, with_taps)
    params = [_get(mod, n) for n in param_names(with_taps)]
    return _WindowSolve.apply(spec, y.contiguous(), feat.contiguous(), *params)


class WinMixFn(torch.autograd.Function):
    """out = sum_g score_g x_g (+ dc) (grr_win_mix) with its HIP reverse (grr_win_bwd_mix)."""

    @staticmethod
    def forward(ctx, x: Tensor, score: Tensor, dc: Optional[Tensor]) -> Tensor:
        ctx.save_for_backward(x, score)
        ctx.has_dc = dc is not None
        return K.win_mix(x, score, dc)

    @staticmethod
    def backward(ctx, gout: Tensor):
        x, score = ctx.saved_tensors
        gout = gout.contiguous()
        gx, gscore = K.win_bwd_mix(gout, x, score)
        return gx, gscore, (gout if ctx.has_dc else None)


class WinEdgeWeightsFn(torch.autograd.Function):
    """(features [B,G,F,H,W], multiM [G,F]) -> (w [B,G,K,H,W], degree [B,G,H,W]): extract_edge_weights
    (grr_win_edge_weights) with its reverse (grr_win_bwd_edge_weights; degree = sum_k w, so its gradient
    joins every edge's)."""

    @staticmethod
    def forward(ctx, delta, f5: Tensor, multiM: Tensor):
        b, g, f, h, w = f5.shape
        feat = f5.reshape(b, g * f, h, w).contiguous()
        wt, deg = K.win_edge_weights(feat, 0, g, f, multiM.contiguous(), delta, with_degree=True)
        ctx.delta, ctx.shape5 = delta, f5.shape
        ctx.save_for_backward(feat, multiM, wt)
        return wt, deg

    @staticmethod
    def backward(ctx, gw: Optional[Tensor], gdeg: Optional[Tensor]):
        feat, multiM, wt = ctx.saved_tensors
        b, g, f, h, w = ctx.shape5
        gwc = torch.zeros_like(wt) if gw is None else gw.contiguous().clone()   # consumed by the reverse
        if gdeg is not None:
            gwc += gdeg.unsqueeze(2)
        gfeat = torch.zeros_like(feat)
        gM = torch.zeros_like(multiM)
        K.win_bwd_edge_weights(feat, 0, g, f, multiM.contiguous(), wt, gwc, ctx.delta, gfeat, gM)
        return None, gfeat.view(ctx.shape5), gM


class WinOperatorFn(torch.autograd.Function):
    """GLRFast.forward (kind "glr": S^T (I - W) S x) or GTVFast.forward (kind "gtv": S^T C^T C S x) on a
    window graph (grr_win_solver mode 3), differentiable in x, the edge weights and the four stats-stencil
    parameters (None: the identity stencil of REF1).  Reverse: _Terms.glr_bwd / gtv_bwd at unit scale."""

    @staticmethod
    def forward(ctx, kind: str, delta, x: Tensor, wt: Tensor, *stencil: Optional[Tensor]):
        b, g, c, h, w = x.shape
        with_taps = stencil[0] is not None
        taps = K.win_taps(*stencil) if with_taps else \
            torch.tensor(K.IDENTITY_TAPS, dtype=torch.float32, device=x.device)
        xc, wc = x.contiguous(), wt.contiguous()
        if kind == "glr":
            out = K.win_apply(xc, delta, g, c, wL=wc, tapsL=taps)
        else:
            out = K.win_apply(xc, delta, g, c, wG=wc, tapsG=taps)
        ctx.kind, ctx.delta, ctx.with_taps = kind, delta, with_taps
        ctx.save_for_backward(xc, wc, taps)
        return out

    @staticmethod
    def backward(ctx, gout: Tensor):
        x, wt, taps = ctx.saved_tensors
        g = x.shape[1]
        one = torch.ones(g, dtype=torch.float32, device=x.device)
        T = _Terms(wt, wt, taps, taps, one, one, torch.zeros_like(one), ctx.delta, g)
        gx = torch.zeros_like(x)
        if ctx.kind == "glr":
            T.glr_bwd(x, gout.contiguous(), 1.0, gx)
            gw, gt = T.gwL, T.gtL
        else:
            T.gtv_bwd(x, gout.contiguous(), 1.0, gx)
            gw, gt = T.gwG, T.gtG
        gst = taps_backward(gt) if ctx.with_taps else (None, None, None, None)
        return (None, None, gx, gw, *gst)
