"""Torch-tensor front end of the HIP kernels (one function per C-ABI entry point).

Every function checks that its tensors are fp32, contiguous and on the GPU,
allocates its outputs with ``torch.empty`` (the C ABI never allocates), and
launches on the current torch stream of that device.  There is no fallback: a CPU
tensor or a missing libgrr.so raises.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import os

import torch

from . import _native
from ._native import Stencil, call

Tensor = torch.Tensor


def _ptr(t: Optional[Tensor]):
    return None if t is None else t.data_ptr()


def _check(name: str, *ts: Optional[Tensor]) -> torch.device:
    dev = None
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError(f"{name}: tensors must be on the GPU (got {t.device}); "
                               "the HIP engine has no CPU path")
        if t.dtype != torch.float32:
            raise TypeError(f"{name}: expected float32, got {t.dtype}")
        if not t.is_contiguous():
            raise ValueError(f"{name}: expected a contiguous tensor")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise RuntimeError(f"{name}: tensors on different devices ({dev} vs {t.device})")
    return dev


def _stream(dev: torch.device):
    return torch.cuda.current_stream(dev).cuda_stream


class LaunchTimer:
    """Brackets each launch with HIP events on the stream it is queued on.

    ``records[kind]`` collects (start, end, algorithmic_bytes) per launch; ``summary()``
    synchronises and returns per-kind launch count, mean duration and achieved GB/s.
    """
    split_lnb = False   # True: C <= 128 LocalNonLinearBlocks timed as "lnb_head" + "lnb_mix"

    def __init__(self):
        self.records = {}

    def run(self, kind: str, nbytes: int, fn, flops: int = 0):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        self.records.setdefault(kind, []).append((s, e, nbytes, flops))

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for kind, recs in self.records.items():
            ms = [s.elapsed_time(e) for s, e, _, _ in recs]
            nb = sum(r[2] for r in recs)
            fl = sum(r[3] for r in recs)
            tot = sum(ms)
            out[kind] = {"launches": len(recs), "total_ms": tot, "mean_ms": tot / len(recs),
                         "bytes_per_launch": nb / len(recs), "gbps": nb / (tot * 1e-3) / 1e9 if tot > 0 else 0.0,
                         "flops_per_launch": fl / len(recs),
                         "tflops": fl / (tot * 1e-3) / 1e12 if tot > 0 else 0.0}
        return out


_TIMER = None


def set_timer(timer):
    """Install (or clear, with None) a LaunchTimer for subsequent launches."""
    global _TIMER
    _TIMER = timer


# GRR_TIMER_SHAPES=1: the instrumented loops time the GEMM-like launches per operand shape
TIMER_SHAPES = os.environ.get("GRR_TIMER_SHAPES", "0") == "1"


def _launch(kind: str, nbytes: int, name: str, *args, flops: int = 0):
    if _TIMER is None:
        call(name, *args)
    else:
        _TIMER.run(kind, int(nbytes), lambda: call(name, *args), int(flops))


def lnb_flops(px: int, c_head: int, c: int, hid: int) -> int:
    """Algorithmic fp32 flops of one LocalNonLinearBlock (REF:911-964) over px pixels: LN (4 per
    input channel), W1 (2 c_head 2hid), depthwise 3x3 (18 per hidden channel), gate (4 per
    gated channel), W2 (2 hid c), skip (3 per output channel)."""
    return px * (4 * c_head + 2 * c_head * 2 * hid + 18 * 2 * hid + 4 * hid + 2 * hid * c + 3 * c)


def stencil(module) -> Stencil:
    """grr_stencil of a GLRFast/GTVFast module (its stats_kernel_p* parameters)."""
    ps = [module.stats_kernel_p01, module.stats_kernel_p02a, module.stats_kernel_p02b, module.stats_kernel_p03]
    _check("stencil", *[p.data for p in ps])
    return Stencil(*[p.data_ptr() for p in ps])


NO_STENCIL = Stencil(None, None, None, None)


# ---------------------------------------------------------------------------
TERM_ROWS = True


def set_term_rows(enable) -> None:
    """Row-streaming (True / 2, default: the LDS-ring row kernel where the shape allows, else the
    register-prefetch one; 1: always the register-prefetch row kernel) or per-pixel (False / 0) term
    reverses (grr_bwd_term_fused)."""
    global TERM_ROWS
    level = 2 if enable is True else int(enable)
    _native.call("grr_bwd_set_term_rows", level)
    TERM_ROWS = level > 0


def set_term_tail(enable: bool) -> None:
    """The wide ring-kernel term reverse's last column strip as a one-column-lane launch (default on)."""
    _native.call("grr_bwd_set_term_tail", int(bool(enable)))


def set_term_acc_max_w(w: int) -> None:
    """Widest image where the LDS-ring term reverse takes the x-gradient pass inside (default 128)."""
    _native.call("grr_bwd_set_term_acc_max_w", int(w))


def term_rows_ok(w: int, f: int) -> bool:
    """Widths / channel counts the row-streaming term reverse takes (16-byte aligned planes assumed)."""
    if w <= 64:
        return f <= 16
    if w <= 128 and w % 2 == 0:
        return f <= 16
    return w % 4 == 0 and f <= 12   # W > 256: column strips


def set_kernel_variant(variant: str) -> None:
    """Select the graph-operator kernels: "auto" (row waves for W <= 256, the channel waves
    of a graph in lockstep), "strips" (column strips at every width) or "independent" (row
    waves, channel waves unsynchronised).  Test / benchmark knob; process-wide."""
    _native.call("grr_set_kernel_variant", {"auto": 0, "strips": 1, "independent": 2}[variant])


def stream_copy(src: Tensor, dst: Tensor) -> None:
    """float4 streaming copy (bench's measured HBM ceiling)."""
    assert src.is_contiguous() and dst.is_contiguous() and src.numel() == dst.numel()
    call("grr_stream_copy", src.data_ptr(), dst.data_ptr(), src.numel(), _stream(src.device))


def neighbor_table(h: int, w: int, device) -> Tensor:
    out = torch.empty((4, h, w), dtype=torch.int32, device=device)
    call("grr_neighbor_table", out.data_ptr(), h, w, _stream(out.device))
    return out


def edge_weights(feat: Tensor, channel_offset: int, n_graphs: int, n_fts: int, multiM: Tensor,
                 with_degree: bool = False) -> Tuple[Tensor, Optional[Tensor]]:
    """Edge weights of the [n_graphs*n_fts] channel slab starting at ``channel_offset`` of feat [B,Ctot,H,W]."""
    dev = _check("edge_weights", feat, multiM)
    b, ctot, h, w = feat.shape
    if channel_offset + n_graphs * n_fts > ctot:
        raise ValueError("edge_weights: channel slab out of range")
    wt = torch.empty((b, n_graphs, 4, h, w), dtype=torch.float32, device=dev)
    deg = torch.empty((b, n_graphs, h, w), dtype=torch.float32, device=dev) if with_degree else None
    base = feat.data_ptr() + channel_offset * h * w * feat.element_size()
    nbytes = 4 * b * h * w * (n_graphs * n_fts + 4 * n_graphs + (n_graphs if with_degree else 0))
    _launch("edge_weights", nbytes, "grr_edge_weights", base, ctot * h * w, multiM.data_ptr(), wt.data_ptr(),
            _ptr(deg), b, n_graphs, n_fts, h, w, _stream(dev))
    return wt, deg


def edge_weights_block(feat: Tensor, n_graphs: int, n_fts: int, multiM_gtv: Tensor,
                       multiM_glr: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    """Both graph modules of a level from one [B, 2C, H, W] feature map (GTV half first, REF:714):
    returns (wG raw [B,G,4,H,W], cG pair [B,G,2,H,W], wL [B,G,4,H,W])."""
    dev = _check("edge_weights_block", feat, multiM_gtv, multiM_glr)
    b, ctot, h, w = feat.shape
    c = n_graphs * n_fts
    if ctot != 2 * c:
        raise ValueError(f"edge_weights_block: expected {2 * c} feature channels, got {ctot}")
    wG = torch.empty((b, n_graphs, 4, h, w), dtype=torch.float32, device=dev)
    wL = torch.empty_like(wG)
    cG = torch.empty((b, n_graphs, 2, h, w), dtype=torch.float32, device=dev)
    nbytes = 4 * b * h * w * (2 * c + 10 * n_graphs)
    _launch("edge_weights", nbytes, "grr_edge_weights_block", feat.data_ptr(), ctot * h * w, 0,
            multiM_gtv.data_ptr(), c, multiM_glr.data_ptr(), wG.data_ptr(), cG.data_ptr(), wL.data_ptr(),
            b, n_graphs, n_fts, h, w, _stream(dev))
    return wG, cG, wL


def feature_edges_ok(c: int, n_graphs: int, n_fts: int, h: int, w: int) -> bool:
    """Where feature_edges applies: grr_feature_edges_supported's conditions (F = 3, G <= 32, C = G F) in plain
    Python (traceable; tests/test_abi.py checks the two agree)."""
    return (n_fts == 3 and 1 <= n_graphs <= 32 and c == n_graphs * n_fts and c <= 96 and h >= 1 and w >= 1
            and n_graphs * 4 * h * w * 4 < (1 << 31) and ((c + 7) // 8) * 8 * h * w * 4 < (1 << 31))


def feature_edges(x: Tensor, x_blocked: bool, weight: Tensor, n_graphs: int, n_fts: int, multiM_gtv: Tensor,
                  multiM_glr: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    """edge_weights_block(conv1x1(x, weight), ...) in one pass (grr_feature_edges): the [B, 2C, H, W]
    features stay on chip.  x: [B, C, H, W], or the channel-blocked layout (x_blocked, lnb_forward_c8's).
    Returns (wG raw [B,G,4,H,W], cG pair [B,G,2,H,W], wL [B,G,4,H,W])."""
    dev = _check("feature_edges", x, weight, multiM_gtv, multiM_glr)
    if x_blocked:
        b, _, h, w, _ = x.shape
        c = n_graphs * n_fts
    else:
        b, c, h, w = x.shape
    if tuple(weight.shape[:2]) != (2 * n_graphs * n_fts, c):
        raise ValueError(f"feature_edges: weight {tuple(weight.shape)} for {c} -> {2 * n_graphs * n_fts} channels")
    wG = torch.empty((b, n_graphs, 4, h, w), dtype=torch.float32, device=dev)
    wL = torch.empty_like(wG)
    cG = torch.empty((b, n_graphs, 2, h, w), dtype=torch.float32, device=dev)
    lib = _native.load()
    ws = torch.empty((lib.grr_feature_edges_workspace_bytes(n_graphs) + 3) // 4, dtype=torch.float32, device=dev)
    nbytes = 4 * b * h * w * (c + 10 * n_graphs)   # x in; wG, wL, cG out
    _launch("feature_edges", nbytes, "grr_feature_edges", x.contiguous().data_ptr(), int(x_blocked),
            weight.contiguous().data_ptr(), multiM_gtv.contiguous().data_ptr(), multiM_glr.contiguous().data_ptr(),
            wG.data_ptr(), cG.data_ptr(), wL.data_ptr(), ws.data_ptr(), b, c, n_graphs, n_fts, h, w, _stream(dev),
            flops=2 * b * h * w * c * 2 * c)
    return wG, cG, wL


def gtv_pair_weights(w: Tensor) -> Tensor:
    dev = _check("gtv_pair_weights", w)
    b, g, four, h, ww = w.shape
    assert four == 4
    c = torch.empty((b, g, 2, h, ww), dtype=torch.float32, device=dev)
    _launch("gtv_pair_weights", 4 * b * g * h * ww * 6, "grr_gtv_pair_weights", w.data_ptr(), c.data_ptr(),
            b, g, h, ww, _stream(dev))
    return c


def pool2(x: Tensor) -> Tensor:
    dev = _check("pool2", x)
    b, c, h, w = x.shape
    out = torch.empty((b, c, h // 2, w // 2), dtype=torch.float32, device=dev)
    _launch("pool2", 4 * b * c * h * w * 5 // 4, "grr_pool2", x.data_ptr(), out.data_ptr(), b, c, h, w, _stream(dev))
    return out


def system_half(xd: Tensor, wL: Optional[Tensor], cG: Optional[Tensor], sL: Stencil, sG: Stencil,
                log_mu: Optional[Tensor], log_ro: Optional[Tensor], n_graphs: int) -> Tensor:
    dev = _check("system_half", xd, wL, cG, log_mu, log_ro)
    b, c, h, w = xd.shape
    t = torch.empty_like(xd)
    nbytes = 4 * b * h * w * (2 * c + (4 * n_graphs if wL is not None else 0) + (2 * n_graphs if cG is not None else 0))
    _launch("system_half", nbytes, "grr_system_half", xd.data_ptr(), _ptr(wL), _ptr(cG), sL, sG, _ptr(log_mu),
            _ptr(log_ro), t.data_ptr(), b, n_graphs, c // n_graphs, h, w, _stream(dev))
    return t


def gtv_rhs_half(xd: Tensor, wG: Tensor, sG: Stencil, prox: bool, log_gamma: Optional[Tensor],
                 n_graphs: int) -> Tensor:
    dev = _check("gtv_rhs_half", xd, wG, log_gamma)
    b, c, h, w = xd.shape
    t = torch.empty_like(xd)
    nbytes = 4 * b * h * w * (2 * c + (4 if prox else 2) * n_graphs)
    _launch("gtv_rhs_half", nbytes, "grr_gtv_rhs_half", xd.data_ptr(), wG.data_ptr(), sG, int(prox),
            _ptr(log_gamma), t.data_ptr(), b, n_graphs, c // n_graphs, h, w, _stream(dev))
    return t


def gtv_rhs_full(x: Tensor, y: Tensor, wG: Tensor, sG: Stencil, prox: bool, log_gamma: Optional[Tensor],
                 log_ro0: Tensor, t_half: Optional[Tensor], log_ro1: Optional[Tensor], n_graphs: int,
                 want_pool: bool = False) -> Tuple[Tensor, Optional[Tensor]]:
    dev = _check("gtv_rhs_full", x, y, wG, log_gamma, log_ro0, t_half, log_ro1)
    b, c, h, w = x.shape
    out = torch.empty_like(x)
    xd = torch.empty((b, c, h // 2, w // 2), dtype=torch.float32, device=dev) if want_pool else None
    px = b * h * w
    nbytes = 4 * (px * (3 * c if x.data_ptr() != y.data_ptr() else 2 * c) + px * (4 if prox else 2) * n_graphs
                  + (px * c // 4 if t_half is not None else 0) + (px * c // 4 if want_pool else 0))
    _launch("gtv_rhs_full", nbytes, "grr_gtv_rhs_full", x.data_ptr(), y.data_ptr(), wG.data_ptr(), sG, int(prox),
            _ptr(log_gamma), log_ro0.data_ptr(), _ptr(t_half), _ptr(log_ro1), out.data_ptr(), _ptr(xd),
            b, n_graphs, c // n_graphs, h, w, _stream(dev))
    return out, xd


def gtv_rhs_full_rep(x: Tensor, x_rep: bool, y: Tensor, y_rep: bool, wG: Tensor, sG: Stencil, prox: bool,
                     log_gamma: Optional[Tensor], log_ro0: Tensor, t_half: Optional[Tensor],
                     log_ro1: Optional[Tensor], n_graphs: int, want_pool: bool = False) -> Tuple[Tensor, Optional[Tensor]]:
    """grr_gtv_rhs_full with x and/or y given as the [B, F, H, W] image they replicate over the graphs."""
    dev = _check("gtv_rhs_full", x, y, wG, log_gamma, log_ro0, t_half, log_ro1)
    full = y if not y_rep else (x if not x_rep else None)
    b, f, h, w = (x if x_rep else y).shape if full is None else (full.shape[0], full.shape[1] // n_graphs,
                                                                  full.shape[2], full.shape[3])
    c = n_graphs * f
    out = torch.empty((b, c, h, w), dtype=torch.float32, device=dev)
    xd = torch.empty((b, c, h // 2, w // 2), dtype=torch.float32, device=dev) if want_pool else None
    px = b * h * w
    nbytes = 4 * (px * (f if x_rep else c) + px * (f if y_rep else c) + px * c + px * (4 if prox else 2) * n_graphs
                  + (px * c // 4 if t_half is not None else 0) + (px * c // 4 if want_pool else 0))
    _launch("gtv_rhs_full", nbytes, "grr_gtv_rhs_full_rep", x.data_ptr(), int(x_rep), y.data_ptr(), int(y_rep),
            wG.data_ptr(), sG, int(prox), _ptr(log_gamma), log_ro0.data_ptr(), _ptr(t_half), _ptr(log_ro1),
            out.data_ptr(), _ptr(xd), b, n_graphs, f, h, w, _stream(dev))
    return out, xd


def system_step(x: Tensor, rhs: Tensor, u_prev: Optional[Tensor], t_half: Optional[Tensor],
                wL: Optional[Tensor], cG: Optional[Tensor], sL: Stencil, sG: Stencil,
                log_mu0: Optional[Tensor], log_ro0: Optional[Tensor], alpha: Tensor, beta: Optional[Tensor],
                n_graphs: int, want_u: bool, want_pool: bool, skip: Optional[Tensor] = None,
                y_skip: Optional[Tensor] = None, u_out: Optional[Tensor] = None) -> Tuple[Tensor, Optional[Tensor], Optional[Tensor]]:
    dev = _check("system_step", x, rhs, u_prev, t_half, wL, cG, log_mu0, log_ro0, alpha, beta, skip, y_skip)
    b, c, h, w = x.shape
    out = torch.empty_like(x)
    if want_u and u_out is None:
        u_out = torch.empty_like(x)
    if not want_u:
        u_out = None
    xd = torch.empty((b, c, h // 2, w // 2), dtype=torch.float32, device=dev) if want_pool else None
    _launch("system_step", step_bytes(b, c, n_graphs, h, w, rhs is not x, u_prev is not None, t_half is not None,
                                      wL is not None, cG is not None, u_out is not None, want_pool, skip is not None),
            "grr_system_step", x.data_ptr(), rhs.data_ptr(), _ptr(u_prev), _ptr(t_half), _ptr(wL), _ptr(cG), sL, sG,
            _ptr(log_mu0), _ptr(log_ro0), alpha.data_ptr(), _ptr(beta), _ptr(skip), _ptr(y_skip),
            out.data_ptr(), _ptr(u_out), _ptr(xd), b, n_graphs, c // n_graphs, h, w, _stream(dev))
    return out, u_out, xd


def system_step2(x: Tensor, rhs: Tensor, u_prev: Optional[Tensor], xd_in: Tensor,
                 wL0: Tensor, cG0: Tensor, sL0: Stencil, sG0: Stencil, log_mu0: Tensor, log_ro0: Tensor,
                 wL1: Tensor, cG1: Tensor, sL1: Stencil, sG1: Stencil, log_mu1: Tensor, log_ro1: Tensor,
                 alpha_a: Tensor, beta_a: Optional[Tensor], alpha_b: Tensor, beta_b: Optional[Tensor],
                 n_graphs: int, want_u: bool, want_pool: bool, skip: Optional[Tensor] = None,
                 y_skip: Optional[Tensor] = None, u_out: Optional[Tensor] = None
                 ) -> Tuple[Tensor, Optional[Tensor], Optional[Tensor]]:
    """Stages k and k+1 in one pass (grr_system_step2), the half level of both inside it; xd_in = D x_k
    (the previous pass's pooled output).  Returns (x_{k+2}, u_{k+2}, D x_{k+2})."""
    dev = _check("system_step2", x, rhs, u_prev, xd_in, wL0, cG0, log_mu0, log_ro0, wL1, cG1, log_mu1, log_ro1,
                 alpha_a, beta_a, alpha_b, beta_b, skip, y_skip)
    b, c, h, w = x.shape
    out = torch.empty_like(x)
    if want_u and (u_out is None or (u_prev is not None and u_out.data_ptr() == u_prev.data_ptr())):
        u_out = torch.empty_like(x)
    if not want_u:
        u_out = None
    xd = torch.empty((b, c, h // 2, w // 2), dtype=torch.float32, device=dev) if want_pool else None
    _launch("system_step2", step2_bytes(b, c, n_graphs, h, w, u_prev is not None, u_out is not None, want_pool,
                                        skip is not None),
            "grr_system_step2", x.data_ptr(), rhs.data_ptr(), _ptr(u_prev), xd_in.data_ptr(), wL0.data_ptr(),
            cG0.data_ptr(), sL0, sG0, log_mu0.data_ptr(), log_ro0.data_ptr(), wL1.data_ptr(), cG1.data_ptr(), sL1, sG1,
            log_mu1.data_ptr(), log_ro1.data_ptr(), alpha_a.data_ptr(), _ptr(beta_a), alpha_b.data_ptr(),
            _ptr(beta_b), _ptr(skip), _ptr(y_skip), out.data_ptr(), _ptr(u_out), _ptr(xd), b, n_graphs,
            c // n_graphs, h, w, _stream(dev))
    return out, u_out, xd


def system_first_pair(b_a: Tensor, xd_a: Tensor, y: Tensor, y_rep: bool,
                      wL0: Tensor, cG0: Tensor, wG0: Tensor, sL0: Stencil, sG0: Stencil, log_mu0: Tensor,
                      log_ro0: Tensor, log_gamma0: Tensor, wL1: Tensor, cG1: Tensor, wG1: Tensor, sL1: Stencil,
                      sG1: Stencil, log_mu1: Tensor, log_ro1: Tensor, log_gamma1: Tensor, alpha0: Tensor,
                      alpha1: Tensor, n_graphs: int) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """Stage 0, the prox right-hand side B and stage 1 in one pass (grr_system_first_pair); xd_a = D b_A.
    y: [B, C, H, W], or the [B, F, H, W] image it replicates (y_rep).  Returns (b_B, x_2, u_2, D x_2)."""
    dev = _check("system_first_pair", b_a, xd_a, y, wL0, cG0, wG0, log_mu0, log_ro0, log_gamma0, wL1, cG1, wG1,
                 log_mu1, log_ro1, log_gamma1, alpha0, alpha1)
    b, c, h, w = b_a.shape
    b_out, x_out, u_out = (torch.empty_like(b_a) for _ in range(3))
    xd = torch.empty((b, c, h // 2, w // 2), dtype=torch.float32, device=dev)
    _launch("system_first_pair", first_pair_bytes(b, c, n_graphs, h, w, y_rep),
            "grr_system_first_pair", b_a.data_ptr(), xd_a.data_ptr(), y.data_ptr(), int(y_rep), wL0.data_ptr(),
            cG0.data_ptr(), wG0.data_ptr(), sL0, sG0, log_mu0.data_ptr(), log_ro0.data_ptr(), log_gamma0.data_ptr(),
            wL1.data_ptr(), cG1.data_ptr(), wG1.data_ptr(), sL1, sG1, log_mu1.data_ptr(), log_ro1.data_ptr(),
            log_gamma1.data_ptr(), alpha0.data_ptr(), alpha1.data_ptr(), b_out.data_ptr(), x_out.data_ptr(),
            u_out.data_ptr(), xd.data_ptr(), b, n_graphs, c // n_graphs, h, w, _stream(dev))
    return b_out, x_out, u_out, xd


def first_pair_bytes(b, c, g, h, w, y_rep):
    """Compulsory HBM bytes of one grr_system_first_pair launch: b_A, D b_A, y read once, the full- and
    half-level GLR + pair weights and the prox raw weights read once per channel group; b_B, x_2, u_2, D x_2
    written once (t_0, x_1, D x_1, the prox terms and t_1 stay on chip)."""
    f = c * (1 + 3) + (c // g if y_rep else c)                         # b_A in; b_B, x_2, u_2 out; y in
    f += (c // 4) * 2                                                  # D b_A in, D x_2 out
    ngrp = -(-(c // g) // 3)
    f += (6 * g + 4 * g + (6 * g + 4 * g) // 4) * ngrp                 # wL0, cG0, wG0; wL1, cG1, wG1
    return 4 * b * h * w * f


# stage 0, right-hand side B and stage 1 in one pass where the shape allows (tests set False for the
# per-stage sequence)
FIRST_PAIR = True


def first_pair_supported(x: Tensor, n_graphs: int) -> bool:
    b, c, h, w = x.shape
    return FIRST_PAIR and w == 256 and h % 2 == 0 and c % n_graphs == 0


# two CG stages per launch where the shape allows (tests set False to run one launch per stage)
STEP2 = True


def system_step2_train(x: Tensor, rhs: Tensor, u_prev: Optional[Tensor], xd_in: Tensor,
                       wL0: Tensor, cG0: Tensor, sL0: Stencil, sG0: Stencil, log_mu0: Tensor, log_ro0: Tensor,
                       wL1: Tensor, cG1: Tensor, sL1: Stencil, sG1: Stencil, log_mu1: Tensor, log_ro1: Tensor,
                       alpha_a: Tensor, beta_a: Optional[Tensor], alpha_b: Tensor, beta_b: Optional[Tensor],
                       n_graphs: int, want_pool: bool, want_mid_pool: bool = False
                       ) -> Tuple[Tensor, Tensor, Tensor, Tensor, Optional[Tensor], Optional[Tensor]]:
    """Stages k, k+1 in one pass keeping the middle iterate (grr_system_step2_train, the training
    forward).  Returns (x_{k+1}, u_{k+1}, x_{k+2}, u_{k+2}, D x_{k+2}, D x_{k+1}); the pooled
    outputs are None unless asked for."""
    dev = _check("system_step2_train", x, rhs, u_prev, xd_in, wL0, cG0, log_mu0, log_ro0, wL1, cG1, log_mu1,
                 log_ro1, alpha_a, beta_a, alpha_b, beta_b)
    b, c, h, w = x.shape
    x_mid, u_mid, out, u_out = (torch.empty_like(x) for _ in range(4))
    xd = torch.empty((b, c, h // 2, w // 2), dtype=torch.float32, device=dev) if want_pool else None
    xdm = torch.empty((b, c, h // 2, w // 2), dtype=torch.float32, device=dev) if want_mid_pool else None
    _launch("system_step2", step2_bytes(b, c, n_graphs, h, w, u_prev is not None, True, want_pool, False)
            + 8 * x.numel() + (x.numel() if want_mid_pool else 0),
            "grr_system_step2_train", x.data_ptr(), rhs.data_ptr(), _ptr(u_prev), xd_in.data_ptr(), wL0.data_ptr(),
            cG0.data_ptr(), sL0, sG0, log_mu0.data_ptr(), log_ro0.data_ptr(), wL1.data_ptr(), cG1.data_ptr(), sL1, sG1,
            log_mu1.data_ptr(), log_ro1.data_ptr(), alpha_a.data_ptr(), _ptr(beta_a), alpha_b.data_ptr(),
            _ptr(beta_b), out.data_ptr(), u_out.data_ptr(), _ptr(xd), x_mid.data_ptr(), u_mid.data_ptr(),
            _ptr(xdm), b, n_graphs, c // n_graphs, h, w, _stream(dev))
    return x_mid, u_mid, out, u_out, xd, xdm


# W != 256 (W % 8 == 0) runs the two-stage pass in column strips of 256 lanes with a 16-column halo
# (STEP2_STRIPS = False: one launch per stage there; bench_wide.py's per-stage comparison).  Narrower images are one strip with idle lanes:
# at W = 128 (the v1.0 model's second level) that still beats one launch per stage (v1.0 forward
# 25.15-25.22 -> 24.75 ms at 16 x 256^2), at W = 64 it does not (25.48 ms; profiles/r03/s2strips/narrow.txt)
STEP2_STRIPS = True
STEP2_MIN_W = 128   # narrowest strip-pass width the loops use


def step2_supported(x: Tensor, n_graphs: int) -> bool:
    """Where the model loops use grr_system_step2: W = 256, or W >= STEP2_MIN_W with W % 8 == 0
    (column strips); even H (F > 3: channel groups of <= 3)."""
    b, c, h, w = x.shape
    wide = STEP2_STRIPS and w >= STEP2_MIN_W and w % 8 == 0
    return (w == 256 or wide) and h % 2 == 0 and c % n_graphs == 0


def step2_bytes(b, c, g, h, w, has_u_prev, has_u_out, has_pool, has_skip):
    """Compulsory HBM bytes of one grr_system_step2 launch: x, b, u_prev, D x_k, the full- and
    half-level GLR + pair weights read once; x_out, u_out, D x_out written once (t_k, x_{k+1},
    u_{k+1}, t_{k+1} stay on chip; the second reads of b rows and of half-level weight rows are
    L2 hits by construction)."""
    f = c * (2 + int(has_u_prev) + 1 + int(has_u_out) + int(has_skip))    # x, b, u_prev, x_out, u_out, y
    f += (c // 4) * (1 + int(has_pool))                                   # D x_k in, D x_out
    ngrp = -(-(c // g) // 3)                                              # workgroups per graph (F > 3)
    f += (6 * g + (6 * g) // 4) * ngrp                                    # full + half-level weights, per group
    return 4 * b * h * w * f


def step_bytes(b, c, g, h, w, has_rhs, has_u_prev, has_half, has_glr, has_gtv, has_u_out, has_pool, has_skip):
    """Compulsory HBM bytes of one grr_system_step launch (each input read once, each output written once)."""
    f = c * (1 + int(has_rhs) + int(has_u_prev) + int(has_u_out) + 1 + int(has_skip))  # x, b, u_prev, u, x_out, y
    f += (c // 4) * (int(has_half) + int(has_pool))                                     # half-level in / out
    f += g * (4 * int(has_glr) + 2 * int(has_gtv))                                      # edge / pair weights
    return 4 * b * h * w * f


# ---- GLRFast / GTVFast sub-API (REF:128-228, :452-516) ---------------------------------
def neighbor_gather(x: Tensor) -> Tensor:
    """get_neighbors_pixels: [B,C,H,W] -> [B,C,4,H,W] replicate-clamped neighbours (REF:128-144)."""
    dev = _check("neighbor_gather", x)
    b, c, h, w = x.shape
    out = torch.empty((b, c, 4, h, w), dtype=torch.float32, device=dev)
    _launch("subapi", 4 * x.numel() * 5, "grr_neighbor_gather", x.data_ptr(), out.data_ptr(), b, c, h, w, _stream(dev))
    return out


def normalize_features(f5: Tensor, multiM: Tensor) -> Tensor:
    """normalize_and_transform_features: [B,G,F,H,W] -> [B,G*F,H,W] (REF:146-157)."""
    dev = _check("normalize_features", f5, multiM)
    b, g, f, h, w = f5.shape
    if tuple(multiM.shape) != (g, f):
        raise ValueError(f"normalize_features: multiM {tuple(multiM.shape)} vs ({g}, {f})")
    out = torch.empty((b, g * f, h, w), dtype=torch.float32, device=dev)
    _launch("subapi", 8 * f5.numel(), "grr_normalize_features", f5.data_ptr(), multiM.data_ptr(), out.data_ptr(),
            b, g, f, h, w, _stream(dev))
    return out


def stats_conv(x5: Tensor, st: Stencil, transpose: bool) -> Tensor:
    """stats_conv (replicate) / stats_conv_transpose (zero frame) of [B,G,F,H,W] (REF:177-215)."""
    dev = _check("stats_conv", x5)
    b, g, f, h, w = x5.shape
    out = torch.empty_like(x5)
    _launch("subapi", 8 * x5.numel(), "grr_stats_conv", x5.data_ptr(), st, int(transpose), out.data_ptr(),
            b, g, f, h, w, _stream(dev))
    return out


def glr_op_L_norm(x5: Tensor, w: Tensor) -> Tensor:
    """GLRFast.op_L_norm: x - sum_e w_e x(clamp(p + delta_e)) (REF:218-228)."""
    dev = _check("glr_op_L_norm", x5, w)
    b, g, f, h, ww = x5.shape
    if tuple(w.shape) != (b, g, 4, h, ww):
        raise ValueError(f"glr_op_L_norm: edge weights {tuple(w.shape)} vs {(b, g, 4, h, ww)}")
    out = torch.empty_like(x5)
    _launch("subapi", 4 * (2 * x5.numel() + w.numel()), "grr_glr_op_l_norm", x5.data_ptr(), w.data_ptr(),
            out.data_ptr(), b, g, f, h, ww, _stream(dev))
    return out


def gtv_op_C(x5: Tensor, w: Tensor, st: Stencil) -> Tensor:
    """GTVFast.op_C: [B,G,F,H,W] -> edge signals [B,G,F,4,H,W] (REF:452-467)."""
    dev = _check("gtv_op_C", x5, w)
    b, g, f, h, ww = x5.shape
    if tuple(w.shape) != (b, g, 4, h, ww):
        raise ValueError(f"gtv_op_C: edge weights {tuple(w.shape)} vs {(b, g, 4, h, ww)}")
    out = torch.empty((b, g, f, 4, h, ww), dtype=torch.float32, device=dev)
    _launch("subapi", 4 * (5 * x5.numel() + w.numel()), "grr_gtv_op_c", x5.data_ptr(), w.data_ptr(), st,
            out.data_ptr(), b, g, f, h, ww, _stream(dev))
    return out


def gtv_op_C_transpose(e6: Tensor, w: Tensor, st: Stencil, want_work: bool = False):
    """GTVFast.op_C_transpose: edge signals [B,G,F,4,H,W] -> [B,G,F,H,W] (REF:469-516)."""
    dev = _check("gtv_op_C_transpose", e6, w)
    b, g, f, four, h, ww = e6.shape
    if four != 4 or tuple(w.shape) != (b, g, 4, h, ww):
        raise ValueError(f"gtv_op_C_transpose: edges {tuple(e6.shape)} / weights {tuple(w.shape)}")
    work = torch.empty((b, g, f, h, ww), dtype=torch.float32, device=dev)
    out = torch.empty_like(work)
    _launch("subapi", 4 * (e6.numel() + w.numel() + 3 * work.numel()), "grr_gtv_op_c_transpose", e6.data_ptr(),
            w.data_ptr(), st, work.data_ptr(), out.data_ptr(), b, g, f, h, ww, _stream(dev))
    return (out, work) if want_work else out


# reverses of the sub-API (csrc/subapi_bwd.hip); gM / gtaps accumulate, gtaps is [G*F, 5]
def neighbor_gather_bwd(g: Tensor) -> Tensor:
    dev = _check("neighbor_gather_bwd", g)
    b, c, four, h, w = g.shape
    gx = torch.empty((b, c, h, w), dtype=torch.float32, device=dev)
    _launch("subapi_bwd", 4 * g.numel() * 5 // 4, "grr_neighbor_gather_bwd", g.data_ptr(), gx.data_ptr(), b, c, h, w,
            _stream(dev))
    return gx


def normalize_features_bwd(f5: Tensor, multiM: Tensor, gout: Tensor, gM: Tensor) -> Tensor:
    dev = _check("normalize_features_bwd", f5, multiM, gout, gM)
    b, g, f, h, w = f5.shape
    gf = torch.empty_like(f5)
    _launch("subapi_bwd", 12 * f5.numel(), "grr_normalize_features_bwd", f5.data_ptr(), multiM.data_ptr(),
            gout.data_ptr(), gf.data_ptr(), gM.data_ptr(), b, g, f, h, w, _stream(dev))
    return gf


def stats_conv_bwd(x5: Tensor, st: Stencil, transpose: bool, g: Tensor, gtaps: Optional[Tensor]) -> Tensor:
    dev = _check("stats_conv_bwd", x5, g, gtaps)
    b, gg, f, h, w = x5.shape
    gx = torch.empty_like(x5)
    _launch("subapi_bwd", 12 * x5.numel(), "grr_stats_conv_bwd", x5.data_ptr(), st, int(transpose), g.data_ptr(),
            gx.data_ptr(), _ptr(gtaps), b, gg, f, h, w, _stream(dev))
    return gx


def glr_op_L_norm_bwd(x5: Tensor, w: Tensor, g: Tensor) -> Tuple[Tensor, Tensor]:
    dev = _check("glr_op_L_norm_bwd", x5, w, g)
    b, gg, f, h, ww = x5.shape
    gx, gw = torch.empty_like(x5), torch.empty_like(w)
    _launch("subapi_bwd", 4 * (3 * x5.numel() + 3 * w.numel()), "grr_glr_op_l_norm_bwd", x5.data_ptr(), w.data_ptr(),
            g.data_ptr(), gx.data_ptr(), gw.data_ptr(), b, gg, f, h, ww, _stream(dev))
    return gx, gw


def gtv_op_C_bwd(x5: Tensor, w: Tensor, st: Stencil, gE: Tensor, gtaps: Tensor) -> Tuple[Tensor, Tensor]:
    dev = _check("gtv_op_C_bwd", x5, w, gE, gtaps)
    b, gg, f, h, ww = x5.shape
    work, gx, gw = torch.empty_like(x5), torch.empty_like(x5), torch.empty_like(w)
    _launch("subapi_bwd", 4 * (gE.numel() + 6 * x5.numel() + 2 * w.numel()), "grr_gtv_op_c_bwd", x5.data_ptr(),
            w.data_ptr(), st, gE.data_ptr(), work.data_ptr(), gx.data_ptr(), gw.data_ptr(), gtaps.data_ptr(),
            b, gg, f, h, ww, _stream(dev))
    return gx, gw


def gtv_op_C_transpose_bwd(e6: Tensor, w: Tensor, st: Stencil, z: Tensor, g: Tensor,
                           gtaps: Tensor) -> Tuple[Tensor, Tensor]:
    dev = _check("gtv_op_C_transpose_bwd", e6, w, z, g, gtaps)
    b, gg, f, four, h, ww = e6.shape
    work2, gE, gw = torch.empty_like(z), torch.empty_like(e6), torch.empty_like(w)
    _launch("subapi_bwd", 4 * (2 * e6.numel() + 4 * z.numel() + 2 * w.numel()), "grr_gtv_op_c_transpose_bwd",
            e6.data_ptr(), w.data_ptr(), st, z.data_ptr(), g.data_ptr(), work2.data_ptr(), gE.data_ptr(),
            gw.data_ptr(), gtaps.data_ptr(), b, gg, f, h, ww, _stream(dev))
    return gE, gw


# ---- feature CNN -----------------------------------------------------------
def conv1x1(x: Tensor, weight: Tensor) -> Tensor:
    """nn.Conv2d(K, M, 1, bias=False) with weight [M,K,1,1]."""
    dev = _check("conv1x1", x, weight)
    b, k, h, w = x.shape
    m = weight.shape[0]
    if weight.shape[1] != k:
        raise ValueError(f"conv1x1: weight {tuple(weight.shape)} vs input channels {k}")
    out = torch.empty((b, m, h, w), dtype=torch.float32, device=dev)
    kind = f"conv1x1[{k}->{m},{b}x{h}x{w}]" if TIMER_SHAPES else "conv1x1"
    ws_bytes = _native.load().grr_conv1x1_workspace_bytes(k, m)
    if ws_bytes > 0:   # split-bf16 MFMA path (fp32-accurate); K > 128 streams K (gemm_x3k_kernel)
        ws = torch.empty((ws_bytes + 3) // 4, dtype=torch.float32, device=dev)  # allocator: 512-B aligned
        _launch(kind, 4 * b * h * w * (k + m), "grr_conv1x1_ws", x.data_ptr(), weight.data_ptr(),
                out.data_ptr(), ws.data_ptr(), b, k, m, h * w, _stream(dev), flops=2 * b * h * w * k * m)
    else:
        _launch(kind, 4 * b * h * w * (k + m), "grr_conv1x1", x.data_ptr(), weight.data_ptr(),
                out.data_ptr(), b, k, m, h * w, _stream(dev), flops=2 * b * h * w * k * m)
    return out


def conv2x2s2(x: Tensor, weight: Tensor) -> Tensor:
    """nn.Conv2d(K, M, 2, stride=2, bias=False) with weight [M,K,2,2]."""
    dev = _check("conv2x2s2", x, weight)
    b, k, h, w = x.shape
    m = weight.shape[0]
    if tuple(weight.shape[1:]) != (k, 2, 2):
        raise ValueError(f"conv2x2s2: weight {tuple(weight.shape)} vs input channels {k}")
    out = torch.empty((b, m, h // 2, w // 2), dtype=torch.float32, device=dev)
    _launch("conv2x2s2", 4 * b * (h * w * k + (h // 2) * (w // 2) * m), "grr_conv2x2s2", x.data_ptr(),
            weight.data_ptr(), out.data_ptr(), b, k, m, h, w, _stream(dev))
    return out


def ffn_forward(x: Tensor, ln_w: Tensor, w_in: Tensor, w_dw: Tensor, w_out: Tensor, skip: Tensor) -> Tensor:
    """FFBlock of the window models' feature CNN (grr_ffn_forward, REF7:13-67): x [B,C,H,W]; ln_w [C];
    w_in [2 hid, C]; w_dw [2 hid, 9]; w_out [C, hid]; skip [2]."""
    dev = _check("ffn_forward", x, ln_w, w_in, w_dw, w_out, skip)
    b, c, h, w = x.shape
    hid = w_out.shape[1]
    if tuple(w_in.shape) != (2 * hid, c) or tuple(w_dw.shape) != (2 * hid, 9) or tuple(w_out.shape) != (c, hid) \
            or ln_w.numel() != c or skip.numel() != 2:
        raise ValueError("ffn_forward: weight shapes disagree with x / hid")
    out = torch.empty_like(x)
    ws = torch.empty((_native.load().grr_ffn_workspace_bytes(b, c, hid, h, w) + 3) // 4, dtype=torch.float32,
                     device=dev)
    p = b * h * w
    _launch("ffn", 4 * p * (2 * c + 3 * hid + 2 * hid), "grr_ffn_forward", x.data_ptr(), ln_w.data_ptr(),
            w_in.data_ptr(), w_dw.data_ptr(), w_out.data_ptr(), skip.data_ptr(), out.data_ptr(), ws.data_ptr(),
            b, c, hid, h, w, _stream(dev), flops=p * (2 * c * 2 * hid + 18 * 2 * hid + 2 * hid * c))
    return out


def wgrad(a: Tensor, bop: Tensor) -> Tensor:
    """Weight gradient out[m, k] = sum_b sum_p a[b, m, p] bop[b, k, p] (grr_wgrad): a [B, M, ...],
    bop [B, K, ...] with the same trailing pixel extent.  The reverse of a 1x1 conv / LNB GEMM's
    weight (REF:556-612 under autograd) without a library GEMM: fp32 MFMA, fixed summation order."""
    dev = _check("wgrad", a, bop)
    b, m = a.shape[:2]
    k = bop.shape[1]
    p = a.numel() // (b * m)
    if bop.shape[0] != b or bop.numel() != b * k * p:
        raise ValueError(f"wgrad: operands {tuple(a.shape)} and {tuple(bop.shape)} disagree")
    out = torch.empty((m, k), dtype=torch.float32, device=dev)
    ws = torch.empty((_native.load().grr_wgrad_workspace_bytes(b, m, k, p) + 3) // 4, dtype=torch.float32,
                     device=dev)
    _launch(f"wgrad[{m}x{k},{b}x{p}]" if TIMER_SHAPES else "wgrad", 4 * b * p * (m + k), "grr_wgrad", a.data_ptr(), bop.data_ptr(), out.data_ptr(), ws.data_ptr(),
            b, m, k, p, _stream(dev), flops=2 * b * p * m * k)
    return out


def set_wgrad_tiles(enable: bool) -> None:
    """grr_wgrad's per-shape wave tile (True, default) or the 128 x 96 tile only (grr_wgrad_set_tiles)."""
    _native.call("grr_wgrad_set_tiles", int(bool(enable)))


_WS_CACHE = {}


# the LNB kernels address one image's [max(hid, C), H, W] planes with 32-bit byte offsets
_LNB_MAX_BYTES = 1 << 31


def _lnb_band_rows(c: int, hid: int, h: int, w: int) -> int:
    """Rows per band so one band (+ its two halo rows) fits the kernels' 32-bit image offsets."""
    per_row = max(hid, c) * w * 4
    return h if per_row * h < _LNB_MAX_BYTES else max(1, (_LNB_MAX_BYTES - 1) // per_row - 2)


def _lnb_banded(run, xs, h: int, rows: int) -> Tensor:
    """Run an LNB forward on row bands of a tall image: the block's only spatial op is the
    depthwise 3x3 (replicate pad), so output rows [r0, r1) need input rows [r0-1, r1+1), and the
    band's own edge padding only reaches the halo rows, which are dropped."""
    outs = []
    for r0 in range(0, h, rows):
        r1 = min(r0 + rows, h)
        a, e = max(r0 - 1, 0), min(r1 + 1, h)
        y = run(*[None if t is None else t[:, :, a:e].contiguous() for t in xs])
        outs.append(y[:, :, r0 - a:r1 - a])
    return torch.cat(outs, 2)


def lnb_forward(x: Tensor, ln_w: Tensor, w1: Tensor, wdw: Tensor, w2: Tensor, skip: Tensor) -> Tensor:
    """LocalNonLinearBlock (nsubnets = 1) forward."""
    dev = _check("lnb_forward", x, ln_w, w1, wdw, w2, skip)
    b, c, h, w = x.shape
    hid = w2.shape[1]
    rows = _lnb_band_rows(c, hid, h, w)
    if rows < h:
        return _lnb_banded(lambda xb: lnb_forward(xb, ln_w, w1, wdw, w2, skip), [x], h, rows)
    lib = _native.load()
    fused = bool(lib.grr_lnb_fused(c, hid))
    # the fused pass needs only its chunk images (g stays on chip); the two-kernel path g + images
    nbytes = lib.grr_lnb_fused_workspace_bytes(c, hid) if fused else lib.grr_lnb_workspace_bytes(b, c, hid, h, w)
    ws = torch.empty((nbytes + 3) // 4, dtype=torch.float32, device=dev)
    out = torch.empty_like(x)
    args = (x.data_ptr(), ln_w.data_ptr(), w1.data_ptr(), wdw.data_ptr(), w2.data_ptr(), skip.data_ptr(),
            out.data_ptr(), ws.data_ptr(), b, c, hid, h, w, _stream(dev))
    if fused:
        # one fused pass (lnb_fused16_kernel): x in (its halo and the skip read once), out written; the
        # gated activation stays on chip
        _launch("lnb_fused", 4 * b * h * w * 2 * c, "grr_lnb_forward", *args, flops=lnb_flops(b * h * w, c, c, hid))
        return out
    if _lnb_split(c):
        _lnb_timed_parts("grr_lnb_forward", args, b * h * w, c, c, hid, c)
        return out
    # C <= 128: x (head), gated g (hid) written and read back once, residual x, out
    nbytes_algo = 4 * b * h * w * (3 * c + 2 * hid) if c <= 128 else 4 * b * h * w * (3 * c + 2 * (2 * hid) + 2 * hid)
    _launch("lnb", nbytes_algo, "grr_lnb_forward", *args, flops=lnb_flops(b * h * w, c, c, hid))
    return out


def c8_shape(b: int, c: int, h: int, w: int) -> Tuple[int, int, int, int, int]:
    """Shape of the channel-blocked layout of a [B, C, H, W] tensor: [B, ceil(C / 8), H, W, 8]."""
    return (b, (c + 7) // 8, h, w, 8)


def to_c8(x: Tensor) -> Tensor:
    """[B, C, H, W] -> the channel-blocked layout (grr_c8_convert; pad channels 0)."""
    dev = _check("to_c8", x)
    b, c, h, w = x.shape
    y = torch.empty(c8_shape(b, c, h, w), dtype=torch.float32, device=dev)
    _launch("c8_convert", 8 * y.numel(), "grr_c8_convert", x.contiguous().data_ptr(), y.data_ptr(), b, c, h, w, 1,
            _stream(dev))
    return y


def from_c8(y: Tensor, c: int) -> Tensor:
    """The channel-blocked layout -> [B, C, H, W]."""
    dev = _check("from_c8", y)
    b, nb, h, w, _ = y.shape
    x = torch.empty((b, c, h, w), dtype=torch.float32, device=dev)
    _launch("c8_convert", 8 * x.numel(), "grr_c8_convert", y.data_ptr(), x.data_ptr(), b, c, h, w, 0, _stream(dev))
    return x


# Python mirror of grr_lnb_set_fused (set_lnb_fused keeps both): the layout decisions below are plain Python so
# that Dynamo traces them (a ctypes query would break the graph); a stale mirror fails loudly in the C entry
# point (GRR_ERR_UNSUPPORTED), never silently
LNB_FUSED = True


def set_lnb_fused(enable: bool) -> None:
    """C <= 96 blocks as one fused pass (default) or on the head + mix kernels (grr_lnb_set_fused)."""
    global LNB_FUSED
    _native.call("grr_lnb_set_fused", int(bool(enable)))
    LNB_FUSED = bool(enable)


def lnb_c8_ok(c: int, hid: int, h: int, w: int) -> bool:
    """Where lnb_forward_c8 applies: the fused C <= 96 pass (grr_lnb_fused), one band."""
    return LNB_FUSED and 2 <= c <= 96 and hid >= 1 and _lnb_band_rows(c, hid, h, w) >= h and \
        ((c + 7) // 8) * 8 * h * w * 4 < (1 << 31)


def lnb_forward_c8(x: Tensor, c: int, ln_w: Tensor, w1: Tensor, wdw: Tensor, w2: Tensor, skip: Tensor,
                   in_c8: bool, out_c8: bool) -> Tensor:
    """lnb_forward with x and / or out in the channel-blocked layout (grr_lnb_forward_c8): a chain of fused
    blocks hands the blocked tensor on, the kernel then loads and stores 16 / 32 bytes per lane instead of
    dwords.  Bitwise equal to lnb_forward.  lnb_c8_ok must hold."""
    dev = _check("lnb_forward_c8", x, ln_w, w1, wdw, w2, skip)
    if in_c8:
        b, _, h, w, _ = x.shape
    else:
        b, c_in, h, w = x.shape
        if c_in != c:
            raise ValueError("lnb_forward_c8: channels")
    hid = w2.shape[1]
    lib = _native.load()
    ws = torch.empty((lib.grr_lnb_fused_workspace_bytes(c, hid) + 3) // 4, dtype=torch.float32, device=dev)
    out = torch.empty(c8_shape(b, c, h, w) if out_c8 else (b, c, h, w), dtype=torch.float32, device=dev)
    xc = x.contiguous()
    _launch("lnb_fused", 4 * b * h * w * 2 * c, "grr_lnb_forward_c8", xc.data_ptr(), ln_w.data_ptr(), w1.data_ptr(),
            wdw.data_ptr(), w2.data_ptr(), skip.data_ptr(), out.data_ptr(), ws.data_ptr(), b, c, hid, h, w,
            int(in_c8) | 2 * int(out_c8), _stream(dev), flops=lnb_flops(b * h * w, c, c, hid))
    return out


def lnb_gate_keepable(c: int, hid: int, h: int, w: int) -> bool:
    """lnb_forward_keep's shapes: the C <= 128 head + mix pipeline in one band (its workspace starts
    with the gated activation g [B, hid, H, W])."""
    return 2 <= c <= 128 and _lnb_band_rows(c, hid, h, w) >= h


def lnb_forward_keep(x: Tensor, ln_w: Tensor, w1: Tensor, wdw: Tensor, w2: Tensor,
                     skip: Tensor) -> Tuple[Tensor, Tensor]:
    """lnb_forward that also returns the head's gated activation g = sigmoid(m) m v,
    [B, hid, H, W] (a view of the launch's workspace), for the training reverse's W2 weight gradient."""
    dev = _check("lnb_forward_keep", x, ln_w, w1, wdw, w2, skip)
    b, c, h, w = x.shape
    hid = w2.shape[1]
    if not lnb_gate_keepable(c, hid, h, w):
        raise ValueError("lnb_forward_keep: needs C <= 128 and one band")
    nbytes = _native.load().grr_lnb_workspace_bytes(b, c, hid, h, w)
    ws = torch.empty((nbytes + 3) // 4, dtype=torch.float32, device=dev)
    out = torch.empty_like(x)
    args = (x.data_ptr(), ln_w.data_ptr(), w1.data_ptr(), wdw.data_ptr(), w2.data_ptr(), skip.data_ptr(),
            out.data_ptr(), ws.data_ptr(), b, c, hid, h, w, _stream(dev))
    if _native.load().grr_lnb_fused(c, hid):
        # the fused pass also stores g (fp32) at the workspace's start: x in, out and g written
        _launch("lnb_fused", 4 * b * h * w * (2 * c + hid), "grr_lnb_forward_keep", *args,
                flops=lnb_flops(b * h * w, c, c, hid))
    elif _lnb_split(c):
        _lnb_timed_parts("grr_lnb_forward_keep", args, b * h * w, c, c, hid, c)
    else:
        _launch("lnb", 4 * b * h * w * (3 * c + 2 * hid), "grr_lnb_forward_keep", *args,
                flops=lnb_flops(b * h * w, c, c, hid))
    return out, ws[:b * hid * h * w].view(b, hid, h, w)


def lnb_forward_rep(src: Tensor, x: Optional[Tensor], ln_w: Tensor, w1: Tensor, wdw: Tensor, w2: Tensor,
                    skip: Tensor) -> Tensor:
    """LocalNonLinearBlock forward when its input [B, R*Cs, H, W] is R copies of src [B, Cs, H, W];
    x is that replicated input (read by the skip) or None (the skip reads src)."""
    dev = _check("lnb_forward_rep", src, x, ln_w, w1, wdw, w2, skip)
    b, cs, h, w = src.shape
    c = ln_w.numel()
    if c % cs or (x is not None and tuple(x.shape) != (b, c, h, w)):
        raise ValueError("lnb_forward_rep: the block input must be copies of src")
    hid = w2.shape[1]
    rows = _lnb_band_rows(c, hid, h, w)
    if rows < h:
        return _lnb_banded(lambda sb, xb: lnb_forward_rep(sb, xb, ln_w, w1, wdw, w2, skip), [src, x], h, rows)
    nbytes = _native.load().grr_lnb_workspace_bytes(b, c, hid, h, w)
    ws = torch.empty((nbytes + 3) // 4, dtype=torch.float32, device=dev)
    out = torch.empty((b, c, h, w), dtype=torch.float32, device=dev)
    args = (src.data_ptr(), cs, c // cs, _ptr(x), ln_w.data_ptr(), w1.data_ptr(), wdw.data_ptr(), w2.data_ptr(),
            skip.data_ptr(), out.data_ptr(), ws.data_ptr(), b, hid, h, w, _stream(dev))
    if _native.load().grr_lnb_rep_fused(cs, c // cs, c, hid):
        # one fused pass (lnb_rep_kernel): src with its 3x3 halo in, out written; no gated tensor in memory
        _launch("lnb_rep_fused", 4 * b * h * w * (cs + 2 * c if x is not None else cs + c), "grr_lnb_forward_rep",
                *args, flops=lnb_flops(b * h * w, cs, c, hid))
        return out
    if _lnb_split(c):
        _lnb_timed_parts("grr_lnb_forward_rep", args, b * h * w, cs, c, hid, c if x is not None else cs)
        return out
    _launch("lnb", 4 * b * h * w * (cs + 2 * c + 2 * hid), "grr_lnb_forward_rep", *args,
            flops=lnb_flops(b * h * w, cs, c, hid))
    return out


# LaunchTimer with split_lnb: the head (LN + W1 + depthwise + gate) and the mix (W2 + skip) of a C <= 128
# block are launched and timed apart on one workspace (grr_lnb_set_phases), as kinds "lnb_head" / "lnb_mix"
def _lnb_split(c: int) -> bool:
    return _TIMER is not None and getattr(_TIMER, "split_lnb", False) and c <= 128


def lnb_head_flops(px: int, c_head: int, hid: int) -> int:
    """Algorithmic fp32 flops of the head: LN (4 per input channel), W1 (2 c_head 2hid), depthwise 3x3
    (18 per hidden channel), gate (4 per gated channel)."""
    return px * (4 * c_head + 2 * c_head * 2 * hid + 18 * 2 * hid + 4 * hid)


def _lnb_timed_parts(name: str, args, px: int, c_head: int, c: int, hid: int, c_skip: int) -> None:
    try:
        call("grr_lnb_set_phases", 3)
        _launch("lnb_head", 4 * px * (c_head + hid), name, *args, flops=lnb_head_flops(px, c_head, hid))
        call("grr_lnb_set_phases", 4)
        _launch("lnb_mix", 4 * px * (hid + c_skip + c), name, *args, flops=px * (2 * hid * c + 3 * c))
    finally:
        call("grr_lnb_set_phases", 7)


def repeat_graphs(img: Tensor, n_graphs: int) -> Tensor:
    dev = _check("repeat_graphs", img)
    b, cin, h, w = img.shape
    out = torch.empty((b, n_graphs * cin, h, w), dtype=torch.float32, device=dev)
    _launch("repeat_graphs", 4 * b * h * w * cin * (1 + n_graphs), "grr_repeat_graphs", img.data_ptr(),
            out.data_ptr(), b, cin, n_graphs, h * w, _stream(dev))
    return out


# ---- reverse pass (training) ------------------------------------------------
# Modes of grr_bwd_stencil / grr_bwd_tapgrad
ST_P, ST_T, ST_T_ADJ, ST_P_ADJ = 0, 1, 2, 3


def stencil_taps(p01: Tensor, p02a: Tensor, p02b: Tensor, p03: Tensor) -> Tensor:
    """[C,5] taps (centre, up, left, right, down) of the 3x3 cross stencil
    p01*k01 + p02a*k02a + p02b*k02b + p03*k03 (REF:56-118, :178-183)."""
    a, b, c, d = (t.reshape(-1) for t in (p01, p02a, p02b, p03))
    return torch.stack([a - b - c + 4 * d, -d, -d, b - d, c - d], dim=1).contiguous()


def stencil_taps_backward(gt: Tensor):
    """Chain [C,5] tap gradients back to (p01, p02a, p02b, p03) gradients, each [C,1,1,1]."""
    dc, du, dl, dr, dd = gt.unbind(1)
    out = (dc, dr - dc, dd - dc, 4 * dc - du - dl - dr - dd)
    return tuple(t.reshape(-1, 1, 1, 1) for t in out)


def _bgfhw(x: Tensor, n_graphs: int):
    b, c, h, w = x.shape
    if c % n_graphs:
        raise ValueError(f"{c} channels not divisible by {n_graphs} graphs")
    return b, n_graphs, c // n_graphs, h, w


def bwd_stencil(x: Tensor, taps: Tensor, mode: int, n_graphs: int, scale: Optional[Tensor] = None,
                out: Optional[Tensor] = None) -> Tensor:
    """out = [out +] scale[g] * mode(x)  (out given -> accumulate)."""
    dev = _check("bwd_stencil", x, taps, scale, out)
    acc = out is not None
    if out is None:
        out = torch.empty_like(x)
    _launch("bwd_stencil", 4 * x.numel() * (3 if acc else 2), "grr_bwd_stencil", x.data_ptr(), taps.data_ptr(), mode,
            _ptr(scale), int(acc), out.data_ptr(), *_bgfhw(x, n_graphs), _stream(dev))
    return out


def padj2_ok(x: Tensor) -> bool:
    return x.shape[3] % 4 == 0


def bwd_padj2(v1: Tensor, taps1: Tensor, scale1: Tensor, v2: Tensor, taps2: Tensor, scale2: Tensor, out: Tensor,
              n_graphs: int) -> None:
    """out += scale1[g] P1*(v1) + scale2[g] P2*(v2) in one pass (the two x-gradient passes of a level's terms)."""
    dev = _check("bwd_padj2", v1, taps1, scale1, v2, taps2, scale2, out)
    _launch("bwd_stencil", 4 * v1.numel() * 4, "grr_bwd_padj2", v1.data_ptr(), taps1.data_ptr(), scale1.data_ptr(),
            v2.data_ptr(), taps2.data_ptr(), scale2.data_ptr(), out.data_ptr(), *_bgfhw(v1, n_graphs), _stream(dev))


def bwd_tapgrad(u: Tensor, z: Tensor, mode: int, n_graphs: int, scale: Optional[Tensor], gtaps: Tensor) -> None:
    dev = _check("bwd_tapgrad", u, z, scale, gtaps)
    _launch("bwd_tapgrad", 8 * u.numel(), "grr_bwd_tapgrad", u.data_ptr(), z.data_ptr(), mode, _ptr(scale),
            gtaps.data_ptr(), *_bgfhw(u, n_graphs), _stream(dev))


def bwd_glr(s: Tensor, a: Tensor, w: Tensor, scale: Tensor, coef: float, gw: Tensor, gdot: Tensor, n_graphs: int):
    dev = _check("bwd_glr", s, a, w, scale, gw, gdot)
    z, ap = torch.empty_like(s), torch.empty_like(s)
    _launch("bwd_glr", 4 * (4 * s.numel() + 3 * w.numel()), "grr_bwd_glr", s.data_ptr(), a.data_ptr(), w.data_ptr(),
            scale.data_ptr(), float(coef), z.data_ptr(), ap.data_ptr(), gw.data_ptr(), _ptr(gdot),
            *_bgfhw(s, n_graphs), _stream(dev))
    return z, ap


def bwd_pair(s: Tensor, a: Tensor, c: Tensor, scale: Tensor, coef: float, gc: Tensor, gdot: Tensor, n_graphs: int):
    dev = _check("bwd_pair", s, a, c, scale, gc, gdot)
    z, ap = torch.empty_like(s), torch.empty_like(s)
    _launch("bwd_pair", 4 * (4 * s.numel() + 3 * c.numel()), "grr_bwd_pair", s.data_ptr(), a.data_ptr(), c.data_ptr(),
            scale.data_ptr(), float(coef), z.data_ptr(), ap.data_ptr(), gc.data_ptr(), _ptr(gdot),
            *_bgfhw(s, n_graphs), _stream(dev))
    return z, ap


def bwd_prox(s: Tensor, a: Tensor, w: Tensor, log_gamma: Tensor, scale: Tensor, coef: float, gw: Tensor,
             ggamma: Tensor, gdot: Tensor, n_graphs: int):
    dev = _check("bwd_prox", s, a, w, log_gamma, scale, gw, ggamma, gdot)
    o, gs = torch.empty_like(s), torch.empty_like(s)
    _launch("bwd_prox", 4 * (4 * s.numel() + 3 * w.numel()), "grr_bwd_prox", s.data_ptr(), a.data_ptr(),
            w.data_ptr(), log_gamma.data_ptr(), scale.data_ptr(), float(coef), o.data_ptr(), gs.data_ptr(),
            gw.data_ptr(), ggamma.data_ptr(), gdot.data_ptr(), *_bgfhw(s, n_graphs), _stream(dev))
    return o, gs


# node-feature counts with a fused reverse instance (measured slower than the multi-pass path
# for F = 6 and 12: 49.6 vs 46.5 ms of term reverses per v1.0 training step at 8 x 256^2)
FUSED_TERM_FTS = (1, 2, 3, 4)
TERM_GLR, TERM_PAIR, TERM_PROX = 0, 1, 2


def bwd_term_fused(mode: int, x: Tensor, g: Tensor, taps: Tensor, w: Tensor, log_gamma: Optional[Tensor],
                   scale: Tensor, coef: float, gw: Tensor, ggamma: Optional[Tensor], gdot: Optional[Tensor],
                   gtaps: Tensor, n_graphs: int) -> Tensor:
    """One-pass reverse of an operator term (grr_bwd_term_fused); returns v for the P* pass."""
    dev = _check("bwd_term_fused", x, g, taps, w, log_gamma, scale, gw, ggamma, gdot, gtaps)
    v = torch.empty_like(x)
    _launch("bwd_term_fused", 4 * (3 * x.numel() + 3 * w.numel()), "grr_bwd_term_fused", mode, x.data_ptr(),
            g.data_ptr(), taps.data_ptr(), w.data_ptr(), _ptr(log_gamma), scale.data_ptr(), float(coef),
            v.data_ptr(), gw.data_ptr(), _ptr(ggamma), _ptr(gdot), gtaps.data_ptr(), *_bgfhw(x, n_graphs),
            _stream(dev))
    return v


def term_acc_ok(mode: int, x: Tensor, n_graphs: int, *planes: Tensor) -> bool:
    """Whether grr_bwd_term_fused_acc takes this term reverse (row kernel with the P* pass inside)."""
    b, c, h, w = x.shape
    if not TERM_ROWS or c % n_graphs or any(t.data_ptr() % 16 for t in (x, *planes)):
        return False
    return bool(_native.load().grr_bwd_term_acc_supported(mode, c // n_graphs, h, w))


def bwd_term_fused_acc(mode: int, x: Tensor, g: Tensor, taps: Tensor, w: Tensor, log_gamma: Optional[Tensor],
                       scale: Tensor, coef: float, gx: Tensor, gw: Tensor, ggamma: Optional[Tensor],
                       gdot: Optional[Tensor], gtaps: Tensor, n_graphs: int) -> None:
    """bwd_term_fused + bwd_stencil(v, taps, ST_P_ADJ, scale, out=gx) in one pass (grr_bwd_term_fused_acc):
    gx += scale[g] P*(v), v never written (term_acc_ok must hold)."""
    dev = _check("bwd_term_fused", x, g, taps, w, log_gamma, scale, gx, gw, ggamma, gdot, gtaps)
    if gx.shape != x.shape:
        raise ValueError(f"bwd_term_fused_acc: gx {tuple(gx.shape)} vs x {tuple(x.shape)}")
    _launch("bwd_term_fused", 4 * (4 * x.numel() + 3 * w.numel()), "grr_bwd_term_fused_acc", mode, x.data_ptr(),
            g.data_ptr(), taps.data_ptr(), w.data_ptr(), _ptr(log_gamma), scale.data_ptr(), float(coef),
            gx.data_ptr(), gw.data_ptr(), _ptr(ggamma), _ptr(gdot), gtaps.data_ptr(), *_bgfhw(x, n_graphs),
            _stream(dev))


def bwd_pair_weights(w: Tensor, gc: Tensor, gw: Tensor) -> None:
    dev = _check("bwd_pair_weights", w, gc, gw)
    b, g, _, h, ww = w.shape
    _launch("bwd_pair_weights", 4 * (3 * w.numel() + gc.numel()), "grr_bwd_pair_weights", w.data_ptr(),
            gc.data_ptr(), gw.data_ptr(), b, g, h, ww, _stream(dev))


def bwd_edge_weights(feat: Tensor, channel_offset: int, n_graphs: int, n_fts: int, multiM: Tensor, w: Tensor,
                     gw: Tensor, gfeat: Tensor, gmultiM: Tensor) -> None:
    """Writes the gradient of the [G*F] slab at channel_offset of gfeat (same shape as feat)."""
    dev = _check("bwd_edge_weights", feat, multiM, w, gw, gfeat, gmultiM)
    b, ctot, h, ww = feat.shape
    if gfeat.shape != feat.shape or channel_offset + n_graphs * n_fts > ctot:
        raise ValueError("bwd_edge_weights: bad slab")
    off = channel_offset * h * ww * 4
    _launch("bwd_edge_weights", 4 * b * h * ww * (2 * n_graphs * n_fts + 8 * n_graphs), "grr_bwd_edge_weights",
            feat.data_ptr() + off, ctot * h * ww, multiM.data_ptr(), w.data_ptr(), gw.data_ptr(),
            gfeat.data_ptr() + off, ctot * h * ww, gmultiM.data_ptr(), b, n_graphs, n_fts, h, ww, _stream(dev))


def bwd_graph_dot(u: Tensor, v: Tensor, out: Tensor, n_graphs: int, coef: float = 1.0) -> None:
    """out[g] += coef * sum over (b, f, pixels) of u * v."""
    dev = _check("bwd_graph_dot", u, v, out)
    _launch("bwd_graph_dot", 8 * u.numel(), "grr_bwd_graph_dot", u.data_ptr(), v.data_ptr(), float(coef),
            out.data_ptr(), *_bgfhw(u, n_graphs), _stream(dev))


def bwd_lincomb(x: Tensor, sa: Optional[Tensor], y: Optional[Tensor], sb: Optional[Tensor], n_graphs: int,
                out: Optional[Tensor] = None, accumulate: bool = False) -> Tensor:
    """out = [out +] sa[g] x + sb[g] y (per-graph coefficient vectors; None = 1)."""
    dev = _check("bwd_lincomb", x, sa, y, sb, out)
    if out is None:
        out = torch.empty_like(x)
        accumulate = False
    _launch("bwd_lincomb", 4 * x.numel() * (2 + int(y is not None) + int(accumulate)), "grr_bwd_lincomb",
            x.data_ptr(), _ptr(sa), _ptr(y), _ptr(sb), out.data_ptr(), int(accumulate), *_bgfhw(x, n_graphs),
            _stream(dev))
    return out


def bwd_cg_glue(gx: Tensor, u: Tensor, gu_next: Optional[Tensor], u_prev: Optional[Tensor], alpha: Tensor,
                beta_next: Optional[Tensor], gbb: Optional[Tensor], galpha: Tensor, gbeta: Optional[Tensor],
                n_graphs: int, inplace: bool = False, gx_half: Optional[Tensor] = None,
                padj: Optional[tuple] = None, want_pool: bool = False):
    """One reverse step of the stage recurrence glue (grr_bwd_cg_glue): returns (gu, gx - gu), and
    D gu third when want_pool (grr_bwd_cg_glue_pool; glue_pool_ok must hold);
    galpha / gbeta accumulate <gx, u> / <gu, u_prev>, gbb += gu.  inplace: gx - gu overwrites gx.
    Passes of the previous stage folded in (gx taken as ((gx + s1 P1*(v1)) + s2 P2*(v2)) + U gx_half):
    padj = (v1, taps1, s1, v2, taps2, s2), bwd_padj2's operands (padj2_ok); gx_half, bwd_unpool2_acc's."""
    v1, t1, s1, v2, t2, s2 = padj if padj is not None else (None,) * 6
    dev = _check("bwd_cg_glue", gx, gx_half, v1, t1, s1, v2, t2, s2, u, gu_next, u_prev, alpha, beta_next, gbb,
                 galpha, gbeta)
    for t in (v1, v2):
        if t is not None and t.shape != gx.shape:
            raise ValueError("bwd_cg_glue: padj shapes")
    for t in (u, gu_next, u_prev, gbb):
        if t is not None and t.shape != gx.shape:
            raise ValueError("bwd_cg_glue: shapes")
    b, c, h, w = gx.shape
    if gx_half is not None and tuple(gx_half.shape) != (b, c, h // 2, w // 2):
        raise ValueError("bwd_cg_glue: gx_half shape")
    gu = torch.empty_like(gx)
    gx_out = gx if inplace else torch.empty_like(gx)
    n_rw = 2 + int(gu_next is not None) + int(u_prev is not None) + 2 * int(gbb is not None) + 2
    n_rw += 2 * int(v1 is not None)
    nbytes = 4 * (gx.numel() * n_rw + (0 if gx_half is None else gx_half.numel()))
    ptrs = (gx.data_ptr(), _ptr(gx_half), _ptr(v1), _ptr(t1), _ptr(s1), _ptr(v2), _ptr(t2), _ptr(s2),
            u.data_ptr(), _ptr(gu_next), _ptr(u_prev), alpha.data_ptr(), _ptr(beta_next), gu.data_ptr(), _ptr(gbb),
            gx_out.data_ptr())
    if want_pool:
        gud = torch.empty((b, c, h // 2, w // 2), dtype=torch.float32, device=dev)
        _launch("bwd_cg_glue", nbytes + gx.numel(), "grr_bwd_cg_glue_pool", *ptrs, gud.data_ptr(),
                galpha.data_ptr(), _ptr(gbeta), *_bgfhw(gx, n_graphs), _stream(dev))
        return gu, gx_out, gud
    _launch("bwd_cg_glue", nbytes, "grr_bwd_cg_glue", *ptrs, galpha.data_ptr(), _ptr(gbeta),
            *_bgfhw(gx, n_graphs), _stream(dev))
    return gu, gx_out


def glue_pool_ok(x: Tensor, *planes: Optional[Tensor], gx_half: Optional[Tensor] = None) -> bool:
    """Where grr_bwd_cg_glue_pool takes the glue: W % 4 == 0, even H, and every operand plane the pass
    reads on its float4 path (x = gx, then u, gu_next, u_prev, gbb, the padj v planes: None = absent)
    16-byte aligned, gx_half 8-byte aligned (the outputs are fresh torch allocations)."""
    b, c, h, w = x.shape
    if w % 4 or h % 2 or any(t is not None and t.data_ptr() % 16 for t in (x, *planes)):
        return False
    return gx_half is None or gx_half.data_ptr() % 8 == 0


def bwd_unpool2_acc(xd: Tensor, out: Tensor) -> None:
    dev = _check("bwd_unpool2_acc", xd, out)
    b, c, h, w = out.shape
    _launch("bwd_unpool2_acc", 4 * (2 * out.numel() + xd.numel()), "grr_bwd_unpool2_acc", xd.data_ptr(),
            out.data_ptr(), b, c, h, w, _stream(dev))


def conv2x2s2_bwd_data_gemm(g: Tensor, weight: Tensor, h: int, w: int) -> Tensor:
    """Data gradient of nn.Conv2d(K, M, 2, stride=2): one split-bf16 1x1 GEMM with the 4K tap rows
    W[m, k, di, dj] -> row (2 di + dj) K + k, then grr_interleave2x2 to full resolution."""
    dev = _check("conv2x2s2_bwd_data", g, weight)
    b, m = g.shape[:2]
    k = weight.shape[1]
    w4 = weight.permute(2, 3, 1, 0).reshape(4 * k, m, 1, 1).contiguous()
    t = conv1x1(g, w4)
    gx = torch.empty((b, k, h, w), dtype=torch.float32, device=dev)
    _launch("interleave2x2", 8 * gx.numel(), "grr_interleave2x2", t.data_ptr(), gx.data_ptr(), b, k, h, w,
            _stream(dev))
    return gx


def conv2x2s2_bwd_data(g: Tensor, weight: Tensor, h: int, w: int) -> Tensor:
    dev = _check("conv2x2s2_bwd_data", g, weight)
    b, m = g.shape[:2]
    k = weight.shape[1]
    gx = torch.empty((b, k, h, w), dtype=torch.float32, device=dev)
    _launch("conv2x2s2_bwd", 4 * (g.numel() + gx.numel()), "grr_conv2x2s2_bwd_data", g.data_ptr(),
            weight.data_ptr(), gx.data_ptr(), b, k, m, h, w, _stream(dev))
    return gx


def glr_stage(x: Tensor, b: Tensor, u_prev: Optional[Tensor], wL: Tensor, sL: Stencil, mu: Tensor, alpha: Tensor,
              beta: Optional[Tensor], n_graphs: int, want_u: bool = True,
              u_out: Optional[Tensor] = None) -> Tuple[Tensor, Optional[Tensor]]:
    """One v10 MixtureGLR stage (grr_glr_stage): returns (x_out, u)."""
    dev = _check("glr_stage", x, b, u_prev, wL, mu, alpha, beta, u_out)
    bb, c, h, w = x.shape
    out = torch.empty_like(x)
    if want_u and u_out is None:
        u_out = torch.empty_like(x)
    if not want_u:
        u_out = None
    nbytes = 4 * bb * h * w * (c * (2 + int(b is not x) + int(u_prev is not None) + int(u_out is not None))
                               + 4 * n_graphs)
    _launch("glr_stage", nbytes, "grr_glr_stage", x.data_ptr(), b.data_ptr(), _ptr(u_prev), wL.data_ptr(), sL,
            mu.data_ptr(), alpha.data_ptr(), _ptr(beta), out.data_ptr(), _ptr(u_out), bb, n_graphs, c // n_graphs,
            h, w, _stream(dev))
    return out, u_out


# ---- LocalNonLinearBlock reverse pieces ---------------------------------------
def lnb_norm(x: Tensor, ln_w: Tensor) -> Tuple[Tensor, Tensor]:
    dev = _check("lnb_norm", x, ln_w)
    b, c, h, w = x.shape
    n = torch.empty_like(x)
    isd = torch.empty((b, h, w), dtype=torch.float32, device=dev)
    _launch("lnb_norm", 8 * x.numel(), "grr_lnb_norm", x.data_ptr(), ln_w.data_ptr(), n.data_ptr(), isd.data_ptr(),
            b, c, h * w, _stream(dev))
    return n, isd


def lnb_norm_bwd(x: Tensor, ln_w: Tensor, isd: Tensor, gn: Tensor, gx: Tensor, gln_w: Tensor) -> None:
    dev = _check("lnb_norm_bwd", x, ln_w, isd, gn, gx, gln_w)
    b, c, h, w = x.shape
    _launch("lnb_norm_bwd", 20 * x.numel(), "grr_lnb_norm_bwd", x.data_ptr(), ln_w.data_ptr(), isd.data_ptr(),
            gn.data_ptr(), gx.data_ptr(), gln_w.data_ptr(), b, c, h * w, _stream(dev))


def lnb_norm_bwd_skip(x: Tensor, ln_w: Tensor, isd: Tensor, gn: Tensor, gout: Tensor, skip: Tensor,
                      gln_w: Tensor, gskip0: Tensor) -> Tensor:
    """The LNB reverse's tail in one pass (grr_lnb_norm_bwd_skip): returns gx = skip[0] gout + d<gn, n>/dx;
    gskip0 += <gout, x>, gln_w += sum gn x isd."""
    dev = _check("lnb_norm_bwd", x, ln_w, isd, gn, gout, skip, gln_w, gskip0)
    b, c, h, w = x.shape
    if gout.shape != x.shape or gn.shape != x.shape:
        raise ValueError("lnb_norm_bwd_skip: shapes")
    gx = torch.empty_like(x)
    _launch("lnb_norm_bwd", 24 * x.numel(), "grr_lnb_norm_bwd_skip", x.data_ptr(), ln_w.data_ptr(), isd.data_ptr(),
            gn.data_ptr(), gout.data_ptr(), skip.data_ptr(), gx.data_ptr(), gln_w.data_ptr(), gskip0.data_ptr(), b, c,
            h * w, _stream(dev))
    return gx


def dwconv3(h: Tensor, wdw: Tensor) -> Tensor:
    dev = _check("dwconv3", h, wdw)
    b, c, hh, ww = h.shape
    out = torch.empty_like(h)
    _launch("dwconv3", 8 * h.numel(), "grr_dwconv3", h.data_ptr(), wdw.data_ptr(), out.data_ptr(), b, c, hh, ww,
            _stream(dev))
    return out


def dwconv3_bwd(g: Tensor, h: Tensor, wdw: Tensor, gwdw: Tensor) -> Tensor:
    dev = _check("dwconv3_bwd", g, h, wdw, gwdw)
    b, c, hh, ww = h.shape
    gh = torch.empty_like(h)
    # compulsory bytes: g and h read once, gh written once (one fused pass for W <= 256)
    _launch("dwconv3_bwd", 12 * h.numel(), "grr_dwconv3_bwd", g.data_ptr(), h.data_ptr(), wdw.data_ptr(), gh.data_ptr(),
            gwdw.data_ptr(), b, c, hh, ww, _stream(dev))
    return gh


def lnb_gate_bwd_scaled(hp: Tensor, gq: Tensor, scale: Tensor, gdot: Tensor) -> Tensor:
    """ghp = scale * (d gate / d hp) . gq;  gdot += <gq, gate>   (grr_lnb_gate_bwd_scaled)."""
    dev = _check("lnb_gate_bwd_scaled", hp, gq, scale, gdot)
    b, c2, h, w = hp.shape
    hid = c2 // 2
    if tuple(gq.shape) != (b, hid, h, w):
        raise ValueError("lnb_gate_bwd_scaled: gq shape")
    ghp = torch.empty_like(hp)
    _launch("lnb_gate", 4 * hp.numel() * 2 + 4 * gq.numel(), "grr_lnb_gate_bwd_scaled", hp.data_ptr(), gq.data_ptr(),
            scale.data_ptr(), ghp.data_ptr(), gdot.data_ptr(), b, hid, h * w, _stream(dev))
    return ghp


def lnb_gate_dw3_ok(h: int, w: int) -> bool:
    """The depthwise / gate row kernels' widths (W > 256: column strips of 4-wide lanes)."""
    return (w <= 64) or (w <= 128 and w % 2 == 0) or (w % 4 == 0)


def set_lnb_bwd_ring(enable: bool) -> None:
    """The LDS-ring gate + depthwise reverse (True, default) or the register row kernel (grr_lnb_set_bwd_ring)."""
    _native.call("grr_lnb_set_bwd_ring", int(bool(enable)))


def lnb_gate_dw3_bwd(hp: Optional[Tensor], gq: Tensor, scale: Tensor, hh: Tensor, wdw: Tensor, gwdw: Tensor,
                     gdot: Tensor) -> Tensor:
    """Gate reverse + depthwise reverse in one row pass (grr_lnb_gate_dw3_bwd): returns gh.
    hp None: the depthwise output is recomputed from hh in-kernel."""
    dev = _check("lnb_gate_dw3_bwd", hp, gq, scale, hh, wdw, gwdw, gdot)
    b, c2, h, w = hh.shape
    if (hp is not None and hp.shape != hh.shape) or tuple(gq.shape) != (b, c2 // 2, h, w):
        raise ValueError("lnb_gate_dw3_bwd: shapes")
    gh = torch.empty_like(hh)
    nbytes = 4 * ((hp.numel() if hp is not None else 0) + gq.numel() + hh.numel() + gh.numel())
    _launch("lnb_gate_dw3_bwd", nbytes, "grr_lnb_gate_dw3_bwd", _ptr(hp), gq.data_ptr(), scale.data_ptr(),
            hh.data_ptr(), wdw.data_ptr(), gh.data_ptr(), gwdw.data_ptr(), gdot.data_ptr(), b, c2 // 2, h, w,
            _stream(dev))
    return gh


def lnb_dw3_gate(hh: Tensor, wdw: Tensor) -> Tensor:
    """gate = sigmoid(m) m v of (m, v) = dwconv3(hh), the depthwise output not stored (grr_lnb_dw3_gate)."""
    dev = _check("lnb_dw3_gate", hh, wdw)
    b, c2, h, w = hh.shape
    gate = torch.empty((b, c2 // 2, h, w), dtype=torch.float32, device=dev)
    _launch("lnb_dw3_gate", 4 * (hh.numel() + gate.numel()), "grr_lnb_dw3_gate", hh.data_ptr(), wdw.data_ptr(),
            gate.data_ptr(), b, c2 // 2, h, w, _stream(dev))
    return gate


def ffn_dw3_gate(hh: Tensor, wdw: Tensor) -> Tensor:
    """gate = gelu(d1) d2 of [d1; d2] = zero-padded dwconv3(hh) (the window FeedForward, REF7:29-48;
    grr_ffn_dw3_gate, the depthwise output not stored)."""
    dev = _check("ffn_dw3_gate", hh, wdw)
    b, c2, h, w = hh.shape
    gate = torch.empty((b, c2 // 2, h, w), dtype=torch.float32, device=dev)
    _launch("ffn_dw3_gate", 4 * (hh.numel() + gate.numel()), "grr_ffn_dw3_gate", hh.data_ptr(), wdw.data_ptr(),
            gate.data_ptr(), b, c2 // 2, h, w, _stream(dev))
    return gate


def ffn_gate_dw3_bwd(gq: Tensor, scale: Tensor, hh: Tensor, wdw: Tensor, gwdw: Tensor, gdot: Tensor) -> Tensor:
    """Reverse of ffn_dw3_gate with the skip scale (grr_ffn_gate_dw3_bwd): returns gh; gwdw += ;
    gdot[0] += <gq, gate>."""
    dev = _check("ffn_gate_dw3_bwd", gq, scale, hh, wdw, gwdw, gdot)
    b, c2, h, w = hh.shape
    if tuple(gq.shape) != (b, c2 // 2, h, w):
        raise ValueError("ffn_gate_dw3_bwd: shapes")
    gh = torch.empty_like(hh)
    _launch("ffn_gate_dw3_bwd", 4 * (gq.numel() + hh.numel() + gh.numel()), "grr_ffn_gate_dw3_bwd", gq.data_ptr(),
            scale.data_ptr(), hh.data_ptr(), wdw.data_ptr(), gh.data_ptr(), gwdw.data_ptr(), gdot.data_ptr(), b,
            c2 // 2, h, w, _stream(dev))
    return gh


def lnb_gate(hp: Tensor, ggate: Optional[Tensor] = None, want_gate: bool = True):
    """gate = sigmoid(m) m v of hp = [m; v]; with ggate also the reverse ghp.  Returns (gate, ghp)."""
    dev = _check("lnb_gate", hp, ggate)
    b, c2, h, w = hp.shape
    hid = c2 // 2
    gate = torch.empty((b, hid, h, w), dtype=torch.float32, device=dev) if want_gate else None
    ghp = torch.empty_like(hp) if ggate is not None else None
    _launch("lnb_gate", 4 * hp.numel() * 2, "grr_lnb_gate", hp.data_ptr(), _ptr(ggate), _ptr(gate), _ptr(ghp), b, hid,
            h * w, _stream(dev))
    return gate, ghp


# ---- window graphs (REF7 = lib/model_GLR_GTV_deep_v7.py, REF1 = lib/model_GLR_GTV_deep_v1.py) ----
_DELTA_CACHE = {}


def _delta_arg(edge_delta) -> Tuple[object, int]:
    """Host int32 [K,2] (dy, dx) array for the window entry points (cached per window)."""
    key = tuple((int(a), int(b)) for a, b in edge_delta)
    arr = _DELTA_CACHE.get(key)
    if arr is None:
        import ctypes
        flat = [v for e in key for v in e]
        arr = (ctypes.c_int32 * len(flat))(*flat)
        _DELTA_CACHE[key] = arr
    return arr, len(key)


def win_edge_weights(feat: Tensor, channel_offset: int, n_graphs: int, n_fts: int, multiM: Tensor, edge_delta,
                     with_degree: bool = False) -> Tuple[Tensor, Optional[Tensor]]:
    """Window-graph edge weights (grr_win_edge_weights, REF7:418-446) of the [n_graphs*n_fts] channel
    slab at ``channel_offset`` of feat [B,Ctot,H,W] -> (w [B,G,K,H,W], degree or None)."""
    dev = _check("win_edge_weights", feat, multiM)
    b, ctot, h, w = feat.shape
    if channel_offset + n_graphs * n_fts > ctot:
        raise ValueError("win_edge_weights: channel slab out of range")
    delta, k = _delta_arg(edge_delta)
    if multiM.numel() != n_graphs * n_fts:
        raise ValueError(f"win_edge_weights: multiM has {multiM.numel()} entries, expected {n_graphs * n_fts}")
    wt = torch.empty((b, n_graphs, k, h, w), dtype=torch.float32, device=dev)
    deg = torch.empty((b, n_graphs, h, w), dtype=torch.float32, device=dev) if with_degree else None
    base = feat.data_ptr() + channel_offset * h * w * feat.element_size()
    nbytes = 4 * b * h * w * (n_graphs * n_fts + k * n_graphs + (n_graphs if with_degree else 0))
    _launch("win_edge_weights", nbytes, "grr_win_edge_weights", base, ctot * h * w, multiM.data_ptr(), delta, k,
            wt.data_ptr(), _ptr(deg), b, n_graphs, n_fts, h, w, _stream(dev))
    return wt, deg


def win_taps(p01: Tensor, p02a: Tensor, p02b: Tensor, p03: Tensor) -> Tensor:
    """(centre, up, left, right, down) of the stats stencil p01 k01 + p02a k02a + p02b k02b + p03 k03
    (REF7:300-358, scalar parameters): centre p01 - p02a - p02b + 4 p03, right p02a - p03,
    down p02b - p03, up = left = -p03."""
    p01, p02a, p02b, p03 = (t.reshape(()) for t in (p01, p02a, p02b, p03))
    return torch.stack([p01 - p02a - p02b + 4.0 * p03, -p03, -p03, p02a - p03, p02b - p03]).float().contiguous()


IDENTITY_TAPS = (1.0, 0.0, 0.0, 0.0, 0.0)


def _check_win_scalars(n_graphs: int, **ts) -> None:
    """Host-side size checks of the per-graph scalars / stencil taps the window kernels index."""
    for name, t in ts.items():
        if t is None:
            continue
        need = 5 if name.startswith("taps") else n_graphs
        if t.numel() < need:
            raise ValueError(f"window graph: {name} has {t.numel()} entries, needs {need}")


def win_solver(mode: int, x: Tensor, y: Tensor, wG: Tensor, tapsG: Tensor, ro: Tensor, edge_delta, n_graphs: int,
               n_sig: int, *, wL: Optional[Tensor] = None, tapsL: Optional[Tensor] = None, mu: Optional[Tensor] = None,
               log_gamma: Optional[Tensor] = None, alpha: Optional[Tensor] = None, beta: Optional[Tensor] = None,
               u_prev: Optional[Tensor] = None, want_u: bool = True,
               pair: bool = False) -> Tuple[Tensor, Optional[Tensor]]:
    """One fused pass of the window-graph MixtureGTV solver (grr_win_solver, REF7:892-1004).
    pair: wG holds win_pair_weights(w_G) (modes 0 and 1: the same linear GTV term from K weights
    per position instead of K plus K gathered reverse-edge weights).

    mode 0: CG step, x [B,G,Fs,H,W], y = rhs [B,G,Fs,H,W] -> (x_next, u);
    mode 1/2: (prox) right-hand side, y [B,Fs,H,W] shared by the graphs, x per graph or
    [B,Fs,H,W] (shared) -> (rhs [B,G,Fs,H,W], None)."""
    dev = _check("win_solver", x, y, wG, tapsG, ro, wL, tapsL, mu, log_gamma, alpha, beta, u_prev)
    delta, k = _delta_arg(edge_delta)
    b, h, w = x.shape[0], x.shape[-2], x.shape[-1]
    x_rep = int(x.dim() == 4)
    if x_rep and x.shape[1] != n_sig or not x_rep and tuple(x.shape[1:3]) != (n_graphs, n_sig):
        raise ValueError(f"win_solver: x has shape {tuple(x.shape)}")
    if tuple(wG.shape) != (b, n_graphs, k, h, w):
        raise ValueError(f"win_solver: wG has shape {tuple(wG.shape)}, expected {(b, n_graphs, k, h, w)}")
    _check_win_scalars(n_graphs, tapsG=tapsG, tapsL=tapsL, ro=ro, mu=mu, log_gamma=log_gamma, alpha=alpha, beta=beta)
    out = torch.empty((b, n_graphs, n_sig, h, w), dtype=torch.float32, device=dev)
    if u_prev is not None and tuple(u_prev.shape) != tuple(out.shape):
        raise ValueError(f"win_solver: u_prev has shape {tuple(u_prev.shape)}, expected {tuple(out.shape)}")
    u_out = torch.empty_like(out) if (mode == 0 and want_u) else None
    planes = b * n_graphs * n_sig
    if mode == 0:
        if tuple(wL.shape) != tuple(wG.shape) or tuple(y.shape) != tuple(out.shape):
            raise ValueError("win_solver: wL / rhs shapes do not match")
        nbytes = 4 * h * w * (planes * (2 + int(u_prev is not None) + 1 + int(u_out is not None))
                              + 2 * k * b * n_graphs)
    else:
        if tuple(y.shape) != (b, n_sig, h, w):
            raise ValueError(f"win_solver: y has shape {tuple(y.shape)}, expected {(b, n_sig, h, w)}")
        nbytes = 4 * h * w * (planes * (1 + int(not x_rep)) + b * n_sig * (1 + x_rep) + k * b * n_graphs)
    if pair and mode == 2:
        raise ValueError("win_solver: the prox rhs (mode 2) needs the raw GTV weights")
    _launch("win_solver", nbytes, "grr_win_solver", mode + (4 if pair else 0), x.data_ptr(), x_rep, y.data_ptr(),
            _ptr(u_prev), _ptr(wL),
            wG.data_ptr(), _ptr(tapsL), tapsG.data_ptr(), _ptr(mu), ro.data_ptr(), _ptr(log_gamma), _ptr(alpha),
            _ptr(beta), delta, k, out.data_ptr(), _ptr(u_out), b, n_graphs, n_sig, h, w, _stream(dev))
    return out, u_out


def win_pair_weights(w: Tensor, edge_delta) -> Tensor:
    """Pair weights c_e(q) = w_e(q)^2 + [q + d_e inside] w_e'(q + d_e)^2 of the linear window GTV
    term (grr_win_pair_weights), w [B,G,K,H,W] -> c of the same shape."""
    dev = _check("win_pair_weights", w)
    delta, k = _delta_arg(edge_delta)
    b, g, kk, h, ww = w.shape
    if kk != k:
        raise ValueError(f"win_pair_weights: w has {kk} edge planes, the window {k}")
    c = torch.empty_like(w)
    _launch("win_pair_weights", 4 * w.numel() * 3, "grr_win_pair_weights", w.data_ptr(), delta, k, c.data_ptr(), b, g,
            h, ww, _stream(dev))
    return c


def win_mix(x: Tensor, score: Tensor, dc: Optional[Tensor] = None) -> Tensor:
    """sum_g x[b,g,c] score[b,g] (+ dc[b,c]) (grr_win_mix, REF7:1006-1009)."""
    dev = _check("win_mix", x, score, dc)
    b, g, c, h, w = x.shape
    if tuple(score.shape) != (b, g, h, w) or (dc is not None and tuple(dc.shape) != (b, c, h, w)):
        raise ValueError("win_mix: score / dc shapes do not match")
    out = torch.empty((b, c, h, w), dtype=torch.float32, device=dev)
    nbytes = 4 * h * w * (x[0].numel() // (h * w) * b + b * g + b * c * (1 + int(dc is not None)))
    _launch("win_mix", nbytes, "grr_win_mix", x.data_ptr(), score.data_ptr(), _ptr(dc), out.data_ptr(), b, g, c, h, w,
            _stream(dev))
    return out


def win_apply(x: Tensor, edge_delta, n_graphs: int, n_sig: int, *, wL: Optional[Tensor] = None,
              tapsL: Optional[Tensor] = None, mu: Optional[Tensor] = None, wG: Optional[Tensor] = None,
              tapsG: Optional[Tensor] = None, ro: Optional[Tensor] = None) -> Tensor:
    """mu S_L^T (I - W_L) S_L x [wL] + ro S_G^T C^T C S_G x [wG] (grr_win_solver mode 3; the
    GLRFast / GTVFast.forward of REF7:503-511, :776-782).  x [B,G,Fs,H,W]."""
    dev = _check("win_apply", x, wL, tapsL, mu, wG, tapsG, ro)
    delta, k = _delta_arg(edge_delta)
    b, g, c, h, w = x.shape
    for t in (wL, wG):
        if t is not None and tuple(t.shape) != (b, n_graphs, k, h, w):
            raise ValueError(f"win_apply: edge weights of shape {tuple(t.shape)}, expected {(b, n_graphs, k, h, w)}")
    if g != n_graphs or c > 3:
        raise ValueError(f"win_apply: x has shape {tuple(x.shape)} (graphs {n_graphs}, at most 3 signal channels)")
    _check_win_scalars(n_graphs, tapsG=tapsG, tapsL=tapsL, ro=ro, mu=mu)
    out = torch.empty_like(x)
    nbytes = 4 * h * w * (2 * x.numel() // (h * w) + k * b * n_graphs * (int(wL is not None) + int(wG is not None)))
    _launch("win_solver", nbytes, "grr_win_solver", 3, x.data_ptr(), 0, None, None, _ptr(wL), _ptr(wG), _ptr(tapsL),
            _ptr(tapsG), _ptr(mu), _ptr(ro), None, None, None, delta, k, out.data_ptr(), None, b, n_graphs, n_sig, h, w,
            _stream(dev))
    return out


# ---- window-graph reverse (window_bwd.hip; training through MixtureGTV of REF7 / REF1) ----
WST_P, WST_T_ADJ, WST_P_ADJ = 0, 1, 2      # S x (reflect) / S^T* g (zero-frame correlation) / S* g
WTAP_P, WTAP_T = 0, 1


def _win5(x: Tensor, n_graphs: int):
    """(B, G, Fs, H, W) of a [B,G,Fs,H,W] window signal."""
    if x.dim() != 5 or x.shape[1] != n_graphs:
        raise ValueError(f"window reverse: expected [B,{n_graphs},Fs,H,W], got {tuple(x.shape)}")
    b, g, fs, h, w = x.shape
    if h < 2 or w < 2:
        raise ValueError("window reverse: the reflect frame needs H, W >= 2")
    return b, g, fs, h, w


def win_bwd_stencil(x: Tensor, taps: Tensor, mode: int, n_graphs: int, scale: Optional[Tensor] = None,
                    out: Optional[Tensor] = None) -> Tensor:
    """out = [out +] scale[g] * mode(x)  (out given -> accumulate)."""
    dev = _check("win_bwd_stencil", x, taps, scale, out)
    dims = _win5(x, n_graphs)
    acc = out is not None
    if out is None:
        out = torch.empty_like(x)
    elif out.shape != x.shape:
        raise ValueError("win_bwd_stencil: out shape")
    _check_win_scalars(n_graphs, taps=taps, scale=scale)
    _launch("win_bwd_stencil", 4 * x.numel() * (2 + int(acc)), "grr_win_bwd_stencil", x.data_ptr(), taps.data_ptr(),
            mode, _ptr(scale), int(acc), out.data_ptr(), *dims, _stream(dev))
    return out


def win_bwd_tapgrad(u: Tensor, z: Tensor, mode: int, n_graphs: int, scale: Optional[Tensor], gtaps: Tensor) -> None:
    dev = _check("win_bwd_tapgrad", u, z, scale, gtaps)
    dims = _win5(u, n_graphs)
    if z.shape != u.shape or gtaps.numel() < 5:
        raise ValueError("win_bwd_tapgrad: shapes")
    _launch("win_bwd_tapgrad", 8 * u.numel(), "grr_win_bwd_tapgrad", u.data_ptr(), z.data_ptr(), mode, _ptr(scale),
            gtaps.data_ptr(), *dims, _stream(dev))


def _edge_shape_ok(w: Tensor, dims, k: int) -> None:
    b, g, _, h, ww = dims
    if tuple(w.shape) != (b, g, k, h, ww):
        raise ValueError(f"window reverse: edge weights of shape {tuple(w.shape)}, expected {(b, g, k, h, ww)}")


# The window term reverses' second pass recomputes the E / PW planes where they are gathered
# (grr_win_bwd_gather_fused) instead of pass 1 writing 2 Fs K floats per pixel for it to read back;
# False: the planes (the A/B and parity reference)
WIN_FUSED_GATHER = True


def win_bwd_glr(s: Tensor, bt: Tensor, w: Tensor, edge_delta, sc: Tensor, coef: float, gw: Tensor,
                gdot: Optional[Tensor], n_graphs: int) -> Tuple[Tensor, Tensor]:
    """GLR term reverse, both passes: returns (l = (I - W) s, gs = (I - W)^T (sc * bt))."""
    dev = _check("win_bwd_glr", s, bt, w, sc, gw, gdot)
    dims = _win5(s, n_graphs)
    delta, k = _delta_arg(edge_delta)
    _edge_shape_ok(w, dims, k)
    if bt.shape != s.shape or gw.shape != w.shape:
        raise ValueError("win_bwd_glr: shapes")
    _check_win_scalars(n_graphs, sc=sc, gdot=gdot)
    b, g, fs, h, ww = dims
    l_out, gs = torch.empty_like(s), torch.empty_like(s)
    if WIN_FUSED_GATHER:   # no E planes: the gather recomputes them (grr_win_bwd_gather_fused)
        _launch("win_bwd_glr", 4 * (4 * s.numel() + 3 * w.numel()), "grr_win_bwd_glr",
                s.data_ptr(), bt.data_ptr(), w.data_ptr(), delta, k, sc.data_ptr(), float(coef), l_out.data_ptr(),
                None, gs.data_ptr(), gw.data_ptr(), _ptr(gdot), *dims, _stream(dev))
        _launch("win_bwd_gather", 4 * (4 * s.numel() + w.numel()), "grr_win_bwd_gather_fused", s.data_ptr(),
                bt.data_ptr(), w.data_ptr(), delta, k, 0, 0, None, sc.data_ptr(), gs.data_ptr(), None, *dims,
                _stream(dev))
        return l_out, gs
    E = torch.empty((b, g, fs, k, h, ww), dtype=torch.float32, device=dev)
    _launch("win_bwd_glr", 4 * (3 * s.numel() + 3 * w.numel() + (k + 2) * s.numel()), "grr_win_bwd_glr",
            s.data_ptr(), bt.data_ptr(), w.data_ptr(), delta, k, sc.data_ptr(), float(coef), l_out.data_ptr(),
            E.data_ptr(), gs.data_ptr(), gw.data_ptr(), _ptr(gdot), *dims, _stream(dev))
    _launch("win_bwd_gather", 4 * (k + 2) * s.numel(), "grr_win_bwd_gather", E.data_ptr(), None, delta, k,
            gs.data_ptr(), None, *dims, _stream(dev))
    return l_out, gs


def win_bwd_gtv(s: Tensor, bt: Tensor, w: Tensor, edge_delta, prox: bool, log_gamma: Optional[Tensor], sc: Tensor,
                coef: float, gw: Tensor, gdot: Optional[Tensor], ggamma: Optional[Tensor],
                n_graphs: int) -> Tuple[Tensor, Tensor]:
    """GTV term (C^T C or C^T phi(C .)) reverse, both passes: returns (o, gs)."""
    dev = _check("win_bwd_gtv", s, bt, w, log_gamma, sc, gw, gdot, ggamma)
    dims = _win5(s, n_graphs)
    delta, k = _delta_arg(edge_delta)
    _edge_shape_ok(w, dims, k)
    if bt.shape != s.shape or gw.shape != w.shape or (prox and log_gamma is None):
        raise ValueError("win_bwd_gtv: shapes / log_gamma")
    _check_win_scalars(n_graphs, sc=sc, gdot=gdot, log_gamma=log_gamma, ggamma=ggamma)
    b, g, fs, h, ww = dims
    o, gs = torch.empty_like(s), torch.empty_like(s)
    if WIN_FUSED_GATHER:   # no E / PW planes: the gather recomputes them (grr_win_bwd_gather_fused)
        _launch("win_bwd_gtv", 4 * (3 * s.numel() + 3 * w.numel()), "grr_win_bwd_gtv",
                s.data_ptr(), bt.data_ptr(), w.data_ptr(), delta, k, int(prox), _ptr(log_gamma), sc.data_ptr(),
                float(coef), None, None, gs.data_ptr(), gw.data_ptr(), _ptr(gdot), _ptr(ggamma), *dims,
                _stream(dev))
        _launch("win_bwd_gather", 4 * (5 * s.numel() + w.numel()), "grr_win_bwd_gather_fused", s.data_ptr(),
                bt.data_ptr(), w.data_ptr(), delta, k, 1, int(prox), _ptr(log_gamma), sc.data_ptr(), gs.data_ptr(),
                o.data_ptr(), *dims, _stream(dev))
        return o, gs
    E = torch.empty((b, g, fs, k, h, ww), dtype=torch.float32, device=dev)
    PW = torch.empty_like(E)
    _launch("win_bwd_gtv", 4 * (3 * s.numel() + 3 * w.numel() + (2 * k + 1) * s.numel()), "grr_win_bwd_gtv",
            s.data_ptr(), bt.data_ptr(), w.data_ptr(), delta, k, int(prox), _ptr(log_gamma), sc.data_ptr(),
            float(coef), PW.data_ptr(), E.data_ptr(), gs.data_ptr(), gw.data_ptr(), _ptr(gdot), _ptr(ggamma), *dims,
            _stream(dev))
    _launch("win_bwd_gather", 4 * (2 * k + 3) * s.numel(), "grr_win_bwd_gather", E.data_ptr(), PW.data_ptr(), delta,
            k, gs.data_ptr(), o.data_ptr(), *dims, _stream(dev))
    return o, gs


def win_bwd_edge_weights(feat: Tensor, channel_offset: int, n_graphs: int, n_fts: int, multiM: Tensor, w: Tensor,
                         gw: Tensor, edge_delta, gfeat: Tensor, gmultiM: Tensor) -> None:
    """Accumulates into the [G*F] slab at channel_offset of gfeat (same shape as feat) and gmultiM;
    gw is consumed (overwritten by the softmax reverse)."""
    dev = _check("win_bwd_edge_weights", feat, multiM, w, gw, gfeat, gmultiM)
    b, ctot, h, ww = feat.shape
    delta, k = _delta_arg(edge_delta)
    if gfeat.shape != feat.shape or channel_offset + n_graphs * n_fts > ctot:
        raise ValueError("win_bwd_edge_weights: bad slab")
    if tuple(w.shape) != (b, n_graphs, k, h, ww) or gw.shape != w.shape or multiM.numel() != n_graphs * n_fts \
            or gmultiM.numel() != n_graphs * n_fts:
        raise ValueError("win_bwd_edge_weights: shapes")
    off = channel_offset * h * ww * 4
    _launch("win_bwd_edge_weights", 4 * b * h * ww * n_graphs * (3 * n_fts + 3 * k), "grr_win_bwd_edge_weights",
            feat.data_ptr() + off, ctot * h * ww, multiM.data_ptr(), w.data_ptr(), gw.data_ptr(), delta, k,
            gfeat.data_ptr() + off, ctot * h * ww, gmultiM.data_ptr(), b, n_graphs, n_fts, h, ww, _stream(dev))


def win_bwd_mix(gout: Tensor, x: Tensor, score: Tensor) -> Tuple[Tensor, Tensor]:
    """Reverse of win_mix: (gx [B,G,Fs,H,W], gscore [B,G,H,W]); gdc = gout."""
    dev = _check("win_bwd_mix", gout, x, score)
    b, g, c, h, w = x.shape
    if tuple(score.shape) != (b, g, h, w) or tuple(gout.shape) != (b, c, h, w):
        raise ValueError("win_bwd_mix: shapes")
    gx, gscore = torch.empty_like(x), torch.empty_like(score)
    _launch("win_bwd_mix", 4 * (2 * x.numel() + 2 * score.numel() + gout.numel()), "grr_win_bwd_mix",
            gout.data_ptr(), x.data_ptr(), score.data_ptr(), gx.data_ptr(), gscore.data_ptr(), b, g, c, h, w,
            _stream(dev))
    return gx, gscore
