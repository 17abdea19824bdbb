"""GLR-only drop-ins of lib/model_GLR_GTV_deep_v10.py (REF10), on the HIP kernels.

``MixtureGLR`` (REF10:241-335): single-scale unrolled GLR solver, features = one 1x1
conv C->C, one graph module, A x = x + mu[g] L x with ``muys00`` stored linearly
(REF10:283-286).  Each unrolled stage is one fused ``grr_glr_stage`` launch (operator +
residual + heavy-ball update); the edge weights are built once.  ``n_cgd_iters`` sets S
(the reference hard-codes 3, REF10:257); S > 3 continues the reference's recurrence.

``LocalLowpassFilteringBlock`` (REF10:394-410) wraps it (no skip in v10).

``GLRImageFilter``: the single-scale GLR-only image-domain filter (config C1 at S = 1):
the image replicated over the G graphs (as REF13:918-921 does for RGB), MixtureGLR, then
a 1x1 projection back.

``MultiScaleMixtureGLR`` / ``MultiScaleGLRImageFilter``: the two-scale GLR-only solver of
config C2 (5-stage multiscale GLR, gray 256x256, G=8 graphs, F=1).

State-dict keys match the reference.  Training: when autograd records, the solver runs
``solver_grad._GLRSolve`` (HIP forward keeping the iterates + HIP reverse sweep).
"""
from __future__ import annotations

import torch
import torch.nn as nn
from torch.nn.parameter import Parameter

from . import ops as OPS
from .compile_backend import HipModule
from . import solver_grad as SG
from .graph_filter import GLRFast, records_grad


class MixtureGLR(HipModule):
    def __init__(self, n_graphs, n_node_fts, alpha_init, beta_init, muy_init, n_cgd_iters: int = 3):
        super().__init__()
        self.n_graphs = n_graphs
        self.n_node_fts = n_node_fts
        self.n_channels = c = n_graphs * n_node_fts
        self.n_cgd_iters = n_cgd_iters
        muy_init = torch.as_tensor(muy_init, dtype=torch.float32)
        self.alphaCGD = Parameter(torch.ones((n_cgd_iters, n_graphs)) * alpha_init)
        self.betaCGD = Parameter(torch.ones((n_cgd_iters, n_graphs)) * beta_init)
        self.patchs_features_extraction = nn.Sequential(nn.Conv2d(c, c, 1, bias=False))
        self.muys00 = Parameter(torch.ones(n_graphs) * muy_init[0])
        self.GLRmodule00 = GLRFast(n_node_fts, n_graphs, M_diag_init=1.0)

    def forward(self, patchs):
        y = patchs.contiguous()
        if y.shape[1] != self.n_channels:
            raise ValueError(f"MixtureGLR: expected {self.n_channels} channels, got {y.shape[1]}")
        if records_grad(self, y):
            return SG.glr_solve(self, y, SG.Conv1x1Fn.apply(y, self.patchs_features_extraction[0].weight))
        return self._solve(y)

    @torch.no_grad()
    def _solve(self, y):
        g, f = self.n_graphs, self.n_node_fts
        feat = OPS.conv1x1(y, self.patchs_features_extraction[0].weight)
        wL, _ = OPS.edge_weights(feat, 0, g, f, self.GLRmodule00.multiM)
        del feat
        mu, alpha, beta = self.muys00, self.alphaCGD, self.betaCGD
        L0 = self.GLRmodule00
        # stage 0: u0 = r0 = y - A y, x1 = y + a0 u0                      (REF10:316-318)
        x, u = OPS.glr_stage(y, y, None, wL, L0, mu, alpha[0], None, g, want_u=self.n_cgd_iters > 1)
        for k in range(1, self.n_cgd_iters):                          # (REF10:320-328)
            x, u = OPS.glr_stage(x, y, u, wL, L0, mu, alpha[k], beta[k], g, want_u=k < self.n_cgd_iters - 1,
                                 u_out=u)
        return x


class LocalLowpassFilteringBlock(HipModule):
    def __init__(self, dim, nsubnets, ngraphs, n_cgd_iters: int = 3):
        super().__init__()
        self.local_filter = MixtureGLR(n_graphs=ngraphs, n_node_fts=dim // ngraphs, alpha_init=0.5, beta_init=0.1,
                                       muy_init=torch.tensor([[0.001], [0.0], [0.0], [0.0]]),
                                       n_cgd_iters=n_cgd_iters)

    def forward(self, x):
        return self.local_filter(x)


class MultiScaleMixtureGLR(HipModule):
    """Two-scale GLR-only unrolled solver (config C2, SURVEY.md §8d: "GLR-only (v10 pattern,
    2 scales)").  The reference has no literal two-scale GLR-only block, so this is the
    v1.0 system operator with its graph-TV terms removed (REF:642-682 without the ro terms),

        A x = x + e^{mu0} L0 x + U(e^{mu1} L1 D x),   L = S^T (I - W) S  (REF:218-237),

    D / U the 2x2 mean pool and its transpose (REF:613, :662-679), driven by the v10 GLR-only
    recurrence (REF10:313-328, b = y throughout since there is no GTV proximal step):
    u_0 = y - A y, x_1 = y + a_0 u_0;  u_k = (y - A x_k) + b_k u_{k-1}, x_{k+1} = x_k + a_k u_k.
    Features follow v10 at full resolution (1x1 C->C, REF10:270-281) and v1.0's half-scale
    branch (2x2/s2 then 1x1, REF:593-612, both C->C here: one graph module per level).
    mu is stored as a log like v1.0 (REF:568-590).  Each stage = one fused half-level launch
    (grr_system_half, GLR only) + one fused full-level launch (grr_system_step, GLR only: A x,
    residual, heavy-ball update and D x_{k+1} for the next stage)."""

    def __init__(self, n_graphs, n_node_fts, alpha_init=0.5, beta_init=0.1, muy_init=((0.001,), (0.0001,)),
                 n_cgd_iters: int = 5):
        super().__init__()
        self.n_graphs = n_graphs
        self.n_node_fts = n_node_fts
        self.n_channels = c = n_graphs * n_node_fts
        self.n_cgd_iters = n_cgd_iters
        muy_init = torch.as_tensor(muy_init, dtype=torch.float32)
        self.alphaCGD = Parameter(torch.ones((n_cgd_iters, n_graphs)) * alpha_init)
        self.betaCGD = Parameter(torch.ones((n_cgd_iters, n_graphs)) * beta_init)
        self.patchs_features_extraction00 = nn.Sequential(nn.Conv2d(c, c, 1, bias=False))
        self.muys00 = Parameter(torch.ones(n_graphs) * torch.log(muy_init[0]))
        self.GLRmodule00 = GLRFast(n_node_fts, n_graphs, M_diag_init=1.0)
        self.patchs_features_extraction01 = nn.Sequential(nn.Conv2d(c, c, 2, stride=2, bias=False),
                                                          nn.Conv2d(c, c, 1, bias=False))
        self.register_buffer("scaling_kernel01", torch.full((c, 1, 2, 2), 0.25), persistent=False)
        self.muys01 = Parameter(torch.ones(n_graphs) * torch.log(muy_init[1]))
        self.GLRmodule01 = GLRFast(n_node_fts, n_graphs, M_diag_init=1.0)

    def forward(self, patchs):
        y = patchs.contiguous()
        b, c, h, w = y.shape
        if c != self.n_channels or h % 2 or w % 2:
            raise ValueError(f"MultiScaleMixtureGLR: expected [B,{self.n_channels},H,W] with even H, W, "
                             f"got {tuple(y.shape)}")
        s0, s1 = self.patchs_features_extraction00, self.patchs_features_extraction01
        if records_grad(self, y):
            f0 = SG.Conv1x1Fn.apply(y, s0[0].weight)
            f1 = SG.Conv1x1Fn.apply(SG.Conv2x2s2Fn.apply(y, s1[0].weight), s1[1].weight)
            return SG.glr2_solve(self, y, f0, f1)
        return self._solve(y)

    @torch.no_grad()
    def _solve(self, y):
        g, f = self.n_graphs, self.n_node_fts
        s0, s1 = self.patchs_features_extraction00, self.patchs_features_extraction01
        f0 = OPS.conv1x1(y, s0[0].weight)
        f1 = OPS.conv1x1(OPS.conv2x2s2(y, s1[0].weight), s1[1].weight)
        wL0, _ = OPS.edge_weights(f0, 0, g, f, self.GLRmodule00.multiM)
        wL1, _ = OPS.edge_weights(f1, 0, g, f, self.GLRmodule01.multiM)
        del f0, f1
        L0, L1 = self.GLRmodule00, self.GLRmodule01
        mu0, mu1 = self.muys00, self.muys01
        alpha, beta = self.alphaCGD, self.betaCGD
        n_st = alpha.shape[0]
        x, u, xd = y, None, OPS.pool2(y)
        for k in range(n_st):                                         # (REF10:316-328)
            last = k == n_st - 1
            t = OPS.system_half(xd, wL1, None, L1, None, mu1, None, g)
            x, u, xd = OPS.system_step(x, y, u, t, wL0, None, L0, None, mu0, None, alpha[k],
                                       beta[k] if k >= 1 else None, g, want_u=not last, want_pool=not last,
                                       u_out=u)
        return x


class MultiScaleGLRImageFilter(HipModule):
    """Config C2 as BASELINE.json states it: the gray image replicated over G graphs
    (as REF13:918-921 does for RGB) -> MultiScaleMixtureGLR (S = 5 two-scale stages) -> 1x1."""

    def __init__(self, n_channels_in=1, n_channels_out=1, ngraphs=8, n_cgd_iters: int = 5):
        super().__init__()
        self.ngraphs = ngraphs
        self.localfilter = MultiScaleMixtureGLR(ngraphs, n_channels_in, n_cgd_iters=n_cgd_iters)
        self.linear_combination = nn.Conv2d(ngraphs * n_channels_in, n_channels_out, 1, bias=False)

    def forward(self, img):
        img = img.contiguous()
        if records_grad(self, img):
            y = self.localfilter(SG.RepeatGraphsFn.apply(img, self.ngraphs))
            return SG.Conv1x1Fn.apply(y.contiguous(), self.linear_combination.weight)
        with torch.no_grad():
            x = OPS.repeat_graphs(img, self.ngraphs)
            return OPS.conv1x1(self.localfilter(x), self.linear_combination.weight)


class GLRImageFilter(HipModule):
    """Single-scale GLR image filter (config C1 with S = 1): image replicated over G graphs ->
    MixtureGLR (S stages) -> 1x1 projection."""

    def __init__(self, n_channels_in=1, n_channels_out=1, ngraphs=8, n_cgd_iters: int = 5):
        super().__init__()
        self.ngraphs = ngraphs
        self.localfilter = MixtureGLR(ngraphs, n_channels_in, 0.5, 0.1, torch.tensor([[0.001], [0.0]]),
                                      n_cgd_iters=n_cgd_iters)
        self.linear_combination = nn.Conv2d(ngraphs * n_channels_in, n_channels_out, 1, bias=False)

    def forward(self, img):
        img = img.contiguous()
        if records_grad(self, img):
            y = self.localfilter(SG.RepeatGraphsFn.apply(img, self.ngraphs))
            return SG.Conv1x1Fn.apply(y.contiguous(), self.linear_combination.weight)
        with torch.no_grad():
            x = OPS.repeat_graphs(img, self.ngraphs)
            return OPS.conv1x1(self.localfilter(x), self.linear_combination.weight)
