"""Multiblock window-graph denoiser of REF1 = exploration/model_multiscale_mixture_GLR/lib/
model_GLR_GTV_deep_v1.py, on the same HIP solver as window_graph.py (REF7).

Differences from REF7 (window_graph.py): the graph modules have no stats stencils
(S = identity, REF1:187-470), the feature CNN is a four-level Restormer-style U-Net
(REF1:108-184), there is no DC estimator (y = the input, REF1:602-676), and
``MultiScaleSequenceDenoiser`` chains three MixtureGTV blocks — 3x3 ring (K = 8) twice, full
5x5 window (K = 24) — each behind a skip mix and a ``SharpeningBlock`` (REF1:768-884), with
6 CG stages (2 before the prox update, 4 after).

Class names, constructor signatures and ``state_dict`` keys match REF1.  Training runs the
solver through ``window_grad`` (HIP forward + HIP reverse, identity stencil: no tap gradients).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
from torch.nn.parameter import Parameter

from . import kernels as K
from .compile_backend import HipModule
from . import window_grad as WG
from .graph_filter import hip_forward, records_grad
from .window_graph import (CONNECTION_FLAGS_3x3, CONNECTION_FLAGS_5x5, Downsample, FFBlock, MixtureGTV as _MixV7,
                           OverlapPatchEmbed, Upsample, window_edges)


class _WindowGraphModuleV1(HipModule):
    """GLRFast / GTVFast of REF1 (:187-221 / :293-340): multiM only, no stats stencil."""

    def __init__(self, n_channels, n_node_fts, n_graphs, connection_window, device=None, M_diag_init=0.4):
        super().__init__()
        self.device = device
        self.n_channels = n_channels
        self.n_node_fts = n_node_fts
        self.n_graphs = n_graphs
        cw = np.asarray(connection_window)
        self.n_edges = int((cw == 1).sum())
        self.connection_window = cw
        self.buffer_size = int(cw.sum())
        self.edge_delta = window_edges(cw)
        self.pad_dim_hw = np.abs(self.edge_delta.min(axis=0))
        self.multiM = Parameter(torch.ones((n_graphs, n_node_fts), device=device) * M_diag_init)
        self._taps = None

    def taps(self) -> torch.Tensor:
        """Identity stencil (1, 0, 0, 0, 0): S x = x exactly."""
        dev = self.multiM.device
        if self._taps is None or self._taps.device != dev:
            self._taps = torch.tensor(K.IDENTITY_TAPS, dtype=torch.float32, device=dev)
        return self._taps

    def _delta(self):
        return tuple((int(a), int(c)) for a, c in self.edge_delta)

    def extract_edge_weights(self, img_features):
        """[B,G,F,H,W] -> (w [B,G,K,H,W], degree [B,G,H,W]) (REF1:255-272); differentiable in the
        features and multiM when autograd records (window_grad.WinEdgeWeightsFn)."""
        if records_grad(self, img_features):
            return WG.WinEdgeWeightsFn.apply(self._delta(), img_features, self.multiM)
        with torch.no_grad():
            b, g, f, h, w = img_features.shape
            feat = img_features.reshape(b, g * f, h, w).contiguous()
            return K.win_edge_weights(feat, 0, g, f, self.multiM.contiguous(), self.edge_delta, with_degree=True)

    def _graph_op(self, kind, patchs, edge_weights):
        if records_grad(self, patchs, edge_weights):   # identity stencil: no tap parameters
            return WG.WinOperatorFn.apply(kind, self._delta(), patchs, edge_weights, None, None, None, None)
        with torch.no_grad():
            b, g, c, h, w = patchs.shape
            if kind == "glr":
                return K.win_apply(patchs.contiguous(), self.edge_delta, g, c, wL=edge_weights.contiguous(),
                                   tapsL=self.taps())
            return K.win_apply(patchs.contiguous(), self.edge_delta, g, c, wG=edge_weights.contiguous(),
                               tapsG=self.taps())


class GLRFast(_WindowGraphModuleV1):
    """x - W x on a window graph (REF1:274-291)."""

    def forward(self, patchs, edge_weights, node_degree=None):
        return self._graph_op("glr", patchs, edge_weights)


class GTVFast(_WindowGraphModuleV1):
    """C^T C, C = W (I - shift) on a window graph (REF1:421-470)."""

    def forward(self, patchs, edge_weights, node_degree=None):
        return self._graph_op("gtv", patchs, edge_weights)


class FeatureExtraction(HipModule):
    """Four-level encoder / decoder of FFBlocks (REF1:108-184); returns the four decoder levels."""

    def __init__(self, inp_channels=3, out_channels=48, dim=48, num_blocks=(1, 2, 2, 4), num_refinement_blocks=4,
                 ffn_expansion_factor=2.66, bias=False):
        super().__init__()

        def blocks(d, n):
            return nn.Sequential(*[FFBlock(d, ffn_expansion_factor, bias) for _ in range(n)])

        self.patch_embed = OverlapPatchEmbed(inp_channels, dim)
        self.encoder_level1 = blocks(dim, num_blocks[0])
        self.down1_2 = Downsample(dim)
        self.encoder_level2 = blocks(dim * 2, num_blocks[1])
        self.down2_3 = Downsample(dim * 2)
        self.encoder_level3 = blocks(dim * 4, num_blocks[2])
        self.down3_4 = Downsample(dim * 4)
        self.latent = blocks(dim * 8, num_blocks[3])
        self.up4_3 = Upsample(dim * 8)
        self.reduce_chan_level3 = nn.Conv2d(dim * 8, dim * 4, kernel_size=1, bias=bias)
        self.decoder_level3 = blocks(dim * 4, num_blocks[2])
        self.up3_2 = Upsample(dim * 4)
        self.reduce_chan_level2 = nn.Conv2d(dim * 4, dim * 2, kernel_size=1, bias=bias)
        self.decoder_level2 = blocks(dim * 2, num_blocks[1])
        self.up2_1 = Upsample(dim * 2)
        self.decoder_level1 = blocks(dim * 2, num_blocks[0])
        self.refinement = blocks(dim * 2, num_refinement_blocks)
        self.output = nn.Conv2d(dim * 2, out_channels, kernel_size=3, stride=1, padding=1, bias=bias)

    def forward(self, inp_img):
        e1 = self.encoder_level1(self.patch_embed(inp_img))
        e2 = self.encoder_level2(self.down1_2(e1))
        e3 = self.encoder_level3(self.down2_3(e2))
        latent = self.latent(self.down3_4(e3))
        d3 = self.decoder_level3(self.reduce_chan_level3(torch.cat([self.up4_3(latent), e3], 1)))
        d2 = self.decoder_level2(self.reduce_chan_level2(torch.cat([self.up3_2(d3), e2], 1)))
        d1 = self.refinement(self.decoder_level1(torch.cat([self.up2_1(d2), e1], 1)))
        return [self.output(d1), d2, d3, latent]


class MixtureGTV(HipModule):
    """REF1:472-676 (n_cgd_iters >= 4; the reference block runs 6)."""

    solve = _MixV7.solve

    def __init__(self, nchannels_in, n_graphs, n_node_fts, connection_window, n_cgd_iters, alpha_init, beta_init,
                 muy_init, ro_init, gamma_init, device=None):
        super().__init__()
        if n_cgd_iters < 4:
            raise ValueError("MixtureGTV: the reference solver runs at least 4 CG stages")
        self.device = device
        self.n_graphs = n_graphs
        self.n_node_fts = n_node_fts
        self.n_total_fts = n_graphs * n_node_fts
        self.n_levels = 4
        self.n_cgd_iters = n_cgd_iters
        self.nchannels_in = nchannels_in
        self.connection_window = connection_window
        muy_init, ro_init, gamma_init = (torch.as_tensor(t, dtype=torch.float32).cpu()
                                         for t in (muy_init, ro_init, gamma_init))
        self.alphaCGD = Parameter(torch.ones((n_cgd_iters, n_graphs), device=device) * alpha_init)
        self.betaCGD = Parameter(torch.ones((n_cgd_iters, n_graphs), device=device) * beta_init)
        self.patchs_features_extraction = FeatureExtraction(
            inp_channels=3, out_channels=self.n_total_fts, dim=self.n_total_fts, num_blocks=[2, 2, 2, 2],
            num_refinement_blocks=4, ffn_expansion_factor=1, bias=False).to(device)
        self.combination_weight = nn.Sequential(
            nn.Conv2d(self.n_total_fts, n_graphs, kernel_size=1, stride=1, padding=0, bias=False),
            nn.Softmax(dim=1)).to(device)
        self.ro00 = Parameter((torch.ones(n_graphs) * ro_init[0]).to(device))
        self.gamma00 = Parameter((torch.ones(n_graphs) * torch.log(gamma_init[0])).to(device))
        self.GTVmodule00 = GTVFast(nchannels_in, n_node_fts, n_graphs, connection_window, device, M_diag_init=1.0)
        self.muys00 = Parameter((torch.ones(n_graphs) * muy_init[0]).to(device))
        self.GLRmodule00 = GLRFast(nchannels_in, n_node_fts, n_graphs, connection_window, device, M_diag_init=1.0)

    def forward(self, patchs):
        if records_grad(self, patchs):          # training: window_grad's HIP forward + reverse
            feats = self.patchs_features_extraction(patchs)[0]
            x = WG.window_solve(self, patchs, feats, with_taps=False)
            return WG.WinMixFn.apply(x, self.combination_weight(feats).contiguous(), None)
        return self._forward_hip(patchs)

    @hip_forward
    def _forward_hip(self, patchs):
        y = patchs.contiguous()
        feats = self.patchs_features_extraction(y)[0].contiguous()
        x = self.solve(y, feats)
        score = self.combination_weight(feats).contiguous()
        return K.win_mix(x, score, None)


class SharpeningBlock(HipModule):
    """s0 x + s1 project_out(gelu(a) b), [a; b] = dwconv(project_in(x)) (REF1:768-787)."""

    def __init__(self, dim_in, dim_out, hidden_features):
        super().__init__()
        self.project_in = nn.Conv2d(dim_in, hidden_features * 2, kernel_size=1, bias=False)
        self.dwconv = nn.Conv2d(hidden_features * 2, hidden_features * 2, kernel_size=3, stride=1, padding=1,
                                groups=hidden_features * 2, bias=False)
        self.project_out = nn.Conv2d(hidden_features, dim_out, kernel_size=1, bias=False)
        self.skip_connect_weight = Parameter(torch.tensor([0.5, 0.5], dtype=torch.float32))

    def forward(self, patchs):
        a, b = self.dwconv(self.project_in(patchs)).chunk(2, dim=1)
        out = self.project_out(nn.functional.gelu(a) * b)
        return self.skip_connect_weight[0] * patchs + self.skip_connect_weight[1] * out


class MultiScaleSequenceDenoiser(HipModule):
    """REF1:790-884: three skip-mixed MixtureGTV blocks, each followed by a SharpeningBlock."""

    def __init__(self, device=None):
        super().__init__()
        self.device = device
        kw = dict(nchannels_in=3, n_graphs=4, n_cgd_iters=6, alpha_init=0.5, beta_init=0.1,
                  muy_init=torch.tensor([[0.1], [0.0], [0.0], [0.0]]), ro_init=torch.tensor([[0.1], [0.0], [0.0], [0.0]]),
                  gamma_init=torch.tensor([[0.001], [0.0], [0.0], [0.0]]), device=device)
        self.skip_connect_weight01 = Parameter(torch.tensor([0.1, 0.9], dtype=torch.float32, device=device))
        self.mixtureGLR_block01 = MixtureGTV(n_node_fts=6, connection_window=CONNECTION_FLAGS_3x3, **kw)
        self.sharp01 = SharpeningBlock(3, 3, 24).to(device)
        self.skip_connect_weight02 = Parameter(torch.tensor([0.1, 0.9], dtype=torch.float32, device=device))
        self.mixtureGLR_block02 = MixtureGTV(n_node_fts=6, connection_window=CONNECTION_FLAGS_3x3, **kw)
        self.sharp02 = SharpeningBlock(3, 3, 24).to(device)
        self.skip_connect_weight03 = Parameter(torch.tensor([0.1, 0.9], dtype=torch.float32, device=device))
        self.mixtureGLR_block03 = MixtureGTV(n_node_fts=12, connection_window=CONNECTION_FLAGS_5x5, **kw)
        self.sharp03 = SharpeningBlock(3, 3, 24).to(device)

    def forward(self, patchs):
        out = self.skip_connect_weight01[0] * patchs + self.skip_connect_weight01[1] * self.mixtureGLR_block01(patchs)
        out = self.sharp01(out)
        out = self.skip_connect_weight02[0] * out + self.skip_connect_weight02[1] * self.mixtureGLR_block02(out)
        out = self.sharp02(out)
        out = self.skip_connect_weight03[0] * out + self.skip_connect_weight03[1] * self.mixtureGLR_block03(out)
        return self.sharp03(out)
