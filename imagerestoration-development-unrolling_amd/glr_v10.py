"""GLR-only drop-ins of lib/model_GLR_GTV_deep_v10.py (REF10), on the HIP kernels.

``MixtureGLR`` (REF10:241-335): single-scale unrolled GLR solver, features = one 1x1
conv C->C, one graph module, A x = x + mu[g] L x with ``muys00`` stored linearly
(REF10:283-286).  Each unrolled stage is one fused ``grr_glr_stage`` launch (operator +
residual + heavy-ball update); the edge weights are built once.  ``n_cgd_iters`` sets S
(the reference hard-codes 3, REF10:257); S > 3 continues the reference's recurrence.

``LocalLowpassFilteringBlock`` (REF10:394-410) wraps it (no skip in v10).

``GLRImageFilter``: the GLR-only image-domain filter of config C2 (SURVEY.md §8d:
5-stage GLR, gray 256x256, G=8 graphs, F=1): the image replicated over the G graphs
(as REF13:918-921 does for RGB), MixtureGLR, then a 1x1 projection back.

State-dict keys match the reference.  Training: when autograd records, the solver runs
``solver_grad._GLRSolve`` (HIP forward keeping the iterates + HIP reverse sweep).
"""
from __future__ import annotations

import torch
import torch.nn as nn
from torch.nn.parameter import Parameter

from . import kernels as K
from . import solver_grad as SG
from .graph_filter import GLRFast, records_grad


class MixtureGLR(nn.Module):
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
        feat = K.conv1x1(y, self.patchs_features_extraction[0].weight.data)
        wL, _ = K.edge_weights(feat, 0, g, f, self.GLRmodule00.multiM.data)
        del feat
        mu, alpha, beta = self.muys00.data, self.alphaCGD.data, self.betaCGD.data
        st = K.stencil(self.GLRmodule00)
        # stage 0: u0 = r0 = y - A y, x1 = y + a0 u0                      (REF10:316-318)
        x, u = K.glr_stage(y, y, None, wL, st, mu, alpha[0], None, g)
        for k in range(1, self.n_cgd_iters):                          # (REF10:320-328)
            x, u = K.glr_stage(x, y, u, wL, st, mu, alpha[k], beta[k], g, want_u=k < self.n_cgd_iters - 1,
                               u_out=u)
        return x


class LocalLowpassFilteringBlock(nn.Module):
    def __init__(self, dim, nsubnets, ngraphs, n_cgd_iters: int = 3):
        super().__init__()
        self.local_filter = MixtureGLR(n_graphs=ngraphs, n_node_fts=dim // ngraphs, alpha_init=0.5, beta_init=0.1,
                                       muy_init=torch.tensor([[0.001], [0.0], [0.0], [0.0]]),
                                       n_cgd_iters=n_cgd_iters)

    def forward(self, x):
        return self.local_filter(x)


class GLRImageFilter(nn.Module):
    """Config C2: image replicated over G graphs -> MixtureGLR (S stages) -> 1x1 projection."""

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
            x = K.repeat_graphs(img, self.ngraphs)
            return K.conv1x1(self.localfilter(x), self.linear_combination.weight.data)
