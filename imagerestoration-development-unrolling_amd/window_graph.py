"""Window-graph image denoisers of the older reference models, on the HIP kernels.

REF7 = exploration/model_multiscale_mixture_GLR/lib/model_GLR_GTV_deep_v7.py.
Its graphs connect every pixel to the K neighbours of a ``connection_window`` (a 0/1
mask; the 5x5 diamond of ``MultiScaleSequenceDenoiser`` gives K = 12, REF7:1032-1038),
and ``MixtureGTV`` runs one ADMM outer update around its CG stages (REF7:936-1011):

    y~ = y - dc(features)                     rhs0 = y~ + ro C^T C y~           (bias 0)
    x = rhs0;  2 CG stages (alpha[0]; alpha[1], beta[1])
    eps = soft(C x, gamma); bias = C x - eps;  rhs1 = y~ + ro C^T (eps - bias)
    x = rhs1;  CG stages 2 .. n_cgd_iters-1
    out = sum_g softmax_g(conv1x1(features))_g x_g + dc

with A = I + mu S_L^T (I - W_L) S_L + ro S_G^T C^T C S_G (S = the module's 3x3 "stats"
stencil with a reflect frame).  Every solver pass is one fused ``grr_win_solver`` launch
(window_ops.hip): the [B,G,F,K,H,W] edge tensors of the reference never exist.  The
feature CNN (``FeatureExtraction``, a small Restormer-style U-Net) and the DC estimator
run on stock PyTorch-ROCm convolutions.

Class names, constructor signatures and ``state_dict`` keys match REF7, so its
checkpoints load unchanged (the ``device`` argument is accepted and used for placement).
Training: when autograd records, ``MixtureGTV`` runs the solver through
``window_grad._WindowSolve`` (HIP forward keeping the iterates + HIP reverse sweep of
window_bwd.hip) and the mixture through ``window_grad.WinMixFn``; the bare GLRFast / GTVFast
calls (``extract_edge_weights``, ``forward``) through ``window_grad.WinEdgeWeightsFn`` /
``WinOperatorFn`` (the same kernels, REF7:418-446, :503-511, :776-782).
"""
from __future__ import annotations

import itertools
from typing import Optional

import numpy as np
import torch
import torch.nn as nn
from torch.nn.parameter import Parameter

from . import kernels as K
from .compile_backend import HipModule
from . import window_grad as WG
from .graph_filter import hip_forward, records_grad

# the linear GTV passes on pair weights (grr_win_pair_weights); False: on the raw directed weights
WIN_PAIR_WEIGHTS = True

CONNECTION_FLAGS_5x5_small = np.array([
    0, 0, 1, 0, 0,
    0, 1, 1, 1, 0,
    1, 1, 0, 1, 1,
    0, 1, 1, 1, 0,
    0, 0, 1, 0, 0,
]).reshape((5, 5))                     # REF7:1032-1038
CONNECTION_FLAGS_3x3 = np.array([1, 1, 1, 1, 0, 1, 1, 1, 1]).reshape((3, 3))   # REF1:795-799
CONNECTION_FLAGS_5x5 = np.ones((5, 5), dtype=np.int64)
CONNECTION_FLAGS_5x5[2, 2] = 0                                                 # REF1:801-807


def window_edges(connection_window) -> np.ndarray:
    """(dy, dx) int32 [K,2] of a 0/1 window mask, in the reference's order (REF7:285-296)."""
    cw = np.asarray(connection_window)
    n = cw.shape[0]
    m = np.arange(n) - n // 2
    delta = np.array(list(itertools.product(m, m)), dtype=np.int32)
    return delta[cw.reshape(-1) == 1]


# ---------------------------------------------------------------------------
# Feature CNN (REF7:13-270): FFBlocks on grr_ffn_forward in inference and on solver_grad.FFNFn (HIP
# forward + reverse) in training; the 3x3 convs (embedding, down / up sampling, output) on stock
# PyTorch-ROCm convolutions
# ---------------------------------------------------------------------------
class CustomLayerNorm(HipModule):
    """x / sqrt(var_c(x) + 1e-5) (unbiased, uncentred), then a per-channel scale (REF7:13-26)."""

    def __init__(self, nchannels):
        super().__init__()
        self.nchannels = nchannels
        self.weighted_transform = nn.Conv2d(nchannels, nchannels, kernel_size=1, stride=1, groups=nchannels,
                                            bias=False)

    def forward(self, x):
        sigma = x.var(dim=1, keepdim=True, correction=1)
        return self.weighted_transform(x / torch.sqrt(sigma + 1e-5))


class FeedForward(HipModule):
    """1x1 -> depthwise 3x3 -> gelu(x1) * x2 -> 1x1 (REF7:29-48)."""

    def __init__(self, dim, ffn_expansion_factor, bias):
        super().__init__()
        hidden = int(dim * ffn_expansion_factor)
        self.project_in = nn.Conv2d(dim, hidden * 2, kernel_size=1, bias=bias)
        self.dwconv = nn.Conv2d(hidden * 2, hidden * 2, kernel_size=3, stride=1, padding=1, groups=hidden * 2,
                                bias=bias)
        self.project_out = nn.Conv2d(hidden, dim, kernel_size=1, bias=bias)

    def forward(self, x):
        x1, x2 = self.dwconv(self.project_in(x)).chunk(2, dim=1)
        return self.project_out(nn.functional.gelu(x1) * x2)


class FFBlock(HipModule):
    """s0 x + s1 FeedForward(norm(x)) (REF7:51-67)."""

    def __init__(self, dim, ffn_expansion_factor, bias):
        super().__init__()
        self.norm = CustomLayerNorm(dim)
        self.skip_connect_weight_final = Parameter(torch.tensor([0.5, 0.5], dtype=torch.float32))
        self.ffn = FeedForward(dim, ffn_expansion_factor, bias)

    def forward(self, x):
        ffn = self.ffn
        if x.is_cuda and ffn.project_in.bias is None and records_grad(self, x) and K.lnb_gate_dw3_ok(*x.shape[2:]):
            # training: HIP forward + HIP reverse (solver_grad.FFNFn)
            from .solver_grad import FFNFn
            return FFNFn.apply(x.contiguous(), self.norm.weighted_transform.weight, ffn.project_in.weight,
                               ffn.dwconv.weight, ffn.project_out.weight, self.skip_connect_weight_final)
        if x.is_cuda and ffn.project_in.bias is None and not records_grad(self, x) \
                and not torch.compiler.is_compiling():
            # inference: the whole block as one grr_ffn_forward (split-bf16 MFMA GEMMs, gelu gate)
            c, hid = x.shape[1], ffn.project_out.weight.shape[1]
            return K.ffn_forward(x.contiguous(), self.norm.weighted_transform.weight.reshape(c).contiguous(),
                                 ffn.project_in.weight.reshape(2 * hid, c).contiguous(),
                                 ffn.dwconv.weight.reshape(2 * hid, 9).contiguous(),
                                 ffn.project_out.weight.reshape(c, hid).contiguous(),
                                 self.skip_connect_weight_final.contiguous())
        # biased variants, rows wider than the row kernels: stock PyTorch-ROCm ops
        return self.skip_connect_weight_final[0] * x + self.skip_connect_weight_final[1] * self.ffn(self.norm(x))


class OverlapPatchEmbed(HipModule):
    def __init__(self, in_c=3, embed_dim=48, bias=False):   # REF7:72-83
        super().__init__()
        self.proj = nn.Conv2d(in_c, embed_dim, kernel_size=3, stride=1, padding=1, bias=bias)

    def forward(self, x):
        return self.proj(x)


class Downsample(HipModule):
    def __init__(self, n_feat):   # REF7:87-100
        super().__init__()
        self.body = nn.Sequential(nn.Conv2d(n_feat, n_feat // 2, kernel_size=3, stride=1, padding=1, bias=False),
                                  nn.PixelUnshuffle(2))

    def forward(self, x):
        return self.body(x)


class Upsample(HipModule):
    def __init__(self, n_feat):   # REF7:102-116
        super().__init__()
        self.body = nn.Sequential(nn.Conv2d(n_feat, n_feat * 2, kernel_size=3, stride=1, padding=1, bias=False),
                                  nn.PixelShuffle(2))

    def forward(self, x):
        return self.body(x)


class FeatureExtraction(HipModule):
    """Two-level encoder / decoder of FFBlocks (REF7:195-270); returns [features]."""

    def __init__(self, inp_channels=3, out_channels=48, dim=48, num_blocks=(1, 2, 2, 4), num_refinement_blocks=4,
                 ffn_expansion_factor=2.66, bias=False):
        super().__init__()
        self.patch_embed = OverlapPatchEmbed(inp_channels, dim)
        self.encoder_level1 = nn.Sequential(*[FFBlock(dim, ffn_expansion_factor, bias) for _ in range(num_blocks[0])])
        self.down1_2 = Downsample(dim)
        self.encoder_level2 = nn.Sequential(*[FFBlock(dim * 2, ffn_expansion_factor, bias)
                                              for _ in range(num_blocks[1])])
        self.up2_1 = Upsample(dim * 2)
        self.decoder_level1 = nn.Sequential(*[FFBlock(dim * 2, ffn_expansion_factor, bias)
                                              for _ in range(num_blocks[0])])
        self.refinement = nn.Sequential(*[FFBlock(dim * 2, ffn_expansion_factor, bias)
                                          for _ in range(num_refinement_blocks)])
        self.output = nn.Conv2d(dim * 2, out_channels, kernel_size=3, stride=1, padding=1, bias=bias)

    def forward(self, inp_img):
        out_enc_level1 = self.encoder_level1(self.patch_embed(inp_img))
        latent = self.encoder_level2(self.down1_2(out_enc_level1))
        inp_dec_level1 = torch.cat([self.up2_1(latent), out_enc_level1], 1)
        out = self.refinement(self.decoder_level1(inp_dec_level1))
        return [self.output(out)]


class DCestimator(HipModule):
    def __init__(self, dim_in, dim_out, hidden_features):   # REF7:785-799
        super().__init__()
        self.project_in = nn.Conv2d(dim_in, hidden_features * 2, kernel_size=1, bias=False)
        self.dwconv = nn.Conv2d(hidden_features * 2, hidden_features * 2, kernel_size=3, stride=1, padding=1,
                                groups=hidden_features * 2, bias=False)
        self.project_out = nn.Conv2d(hidden_features, dim_out, kernel_size=1, bias=False)

    def forward(self, patchs):
        out01, out02 = self.dwconv(self.project_in(patchs)).chunk(2, dim=1)
        return self.project_out(nn.functional.gelu(out01) * out02)


# ---------------------------------------------------------------------------
# Window graph modules (REF7:274-782)
# ---------------------------------------------------------------------------
class _WindowGraphModule(HipModule):
    """Parameters of GLRFast / GTVFast (REF7:274-371 / :514-611): scalar stats-stencil
    weights (p01 1.0, p02a/p02b/p03 0.5) and multiM [G,F]."""

    def __init__(self, n_channels, n_node_fts, n_graphs, connection_window, device=None, M_diag_init=0.4):
        super().__init__()
        self.n_channels = n_channels
        self.n_node_fts = n_node_fts
        self.n_graphs = n_graphs
        cw = np.asarray(connection_window)
        self.n_edges = int((cw == 1).sum())
        self.connection_window = cw
        self.buffer_size = int(cw.sum())
        self.edge_delta = window_edges(cw)
        self.pad_dim_hw = np.abs(self.edge_delta.min(axis=0))
        self.stats_kernel_p01 = Parameter(torch.ones(1, device=device) * 1.0)
        self.stats_kernel_p02a = Parameter(torch.ones(1, device=device) * 0.5)
        self.stats_kernel_p02b = Parameter(torch.ones(1, device=device) * 0.5)
        self.stats_kernel_p03 = Parameter(torch.ones(1, device=device) * 0.5)
        self.multiM = Parameter(torch.ones((n_graphs, n_node_fts), device=device) * M_diag_init)

    def taps(self) -> torch.Tensor:
        """(centre, up, left, right, down) of the stats stencil (REF7:449-467)."""
        return K.win_taps(self.stats_kernel_p01.data, self.stats_kernel_p02a.data, self.stats_kernel_p02b.data,
                          self.stats_kernel_p03.data)

    def _delta(self):
        return tuple((int(a), int(c)) for a, c in self.edge_delta)

    def _stencil(self):
        return (self.stats_kernel_p01, self.stats_kernel_p02a, self.stats_kernel_p02b, self.stats_kernel_p03)

    def extract_edge_weights(self, img_features):
        """[B,G,F,H,W] -> (w [B,G,K,H,W], degree [B,G,H,W]) (REF7:432-446); differentiable in the
        features and multiM when autograd records."""
        if records_grad(self, img_features):
            return WG.WinEdgeWeightsFn.apply(self._delta(), img_features, self.multiM)
        with torch.no_grad():
            b, g, f, h, w = img_features.shape
            feat = img_features.reshape(b, g * f, h, w).contiguous()
            return K.win_edge_weights(feat, 0, g, f, self.multiM.contiguous(), self.edge_delta, with_degree=True)

    def _graph_op(self, kind, patchs, edge_weights):
        if records_grad(self, patchs, edge_weights):
            return WG.WinOperatorFn.apply(kind, self._delta(), patchs, edge_weights, *self._stencil())
        with torch.no_grad():
            b, g, c, h, w = patchs.shape
            if kind == "glr":
                return K.win_apply(patchs.contiguous(), self.edge_delta, g, c, wL=edge_weights.contiguous(),
                                   tapsL=self.taps())
            return K.win_apply(patchs.contiguous(), self.edge_delta, g, c, wG=edge_weights.contiguous(),
                               tapsG=self.taps())


class GLRFast(_WindowGraphModule):
    """S^T (I - W) S on a window graph (REF7:274-511)."""

    def forward(self, patchs, edge_weights, node_degree=None):
        return self._graph_op("glr", patchs, edge_weights)


class GTVFast(_WindowGraphModule):
    """C^T C with C = W (S - S shifted) on a window graph (REF7:514-782)."""

    def forward(self, patchs, edge_weights, node_degree=None):
        return self._graph_op("gtv", patchs, edge_weights)


class MixtureGTV(HipModule):
    """REF7:802-1016.  n_cgd_iters >= 4: two CG stages before the prox update, the rest after
    (the reference indexes rows 0..3; rows past 3 continue the same recurrence)."""

    def __init__(self, nchannels_in, n_graphs, n_node_fts, n_cnn_fts, connection_window, n_cgd_iters, alpha_init,
                 beta_init, muy_init, ro_init, gamma_init, device=None):
        super().__init__()
        if n_cgd_iters < 4:
            raise ValueError("MixtureGTV: the reference solver runs 4 CG stages (n_cgd_iters >= 4)")
        self.device = device
        self.n_graphs = n_graphs
        self.n_node_fts = n_node_fts
        self.n_total_fts = n_graphs * n_node_fts
        self.n_cnn_fts = n_cnn_fts
        self.n_levels = 4
        self.n_cgd_iters = n_cgd_iters
        self.nchannels_in = nchannels_in
        self.connection_window = connection_window
        muy_init, ro_init, gamma_init = (torch.as_tensor(t, dtype=torch.float32).cpu()
                                         for t in (muy_init, ro_init, gamma_init))
        self.alphaCGD = Parameter(torch.ones((n_cgd_iters, n_graphs), device=device) * alpha_init)
        self.betaCGD = Parameter(torch.ones((n_cgd_iters, n_graphs), device=device) * beta_init)
        self.patchs_features_extraction = FeatureExtraction(
            inp_channels=3, out_channels=self.n_total_fts + 12, dim=n_cnn_fts, num_blocks=[4, 3, 3],
            num_refinement_blocks=4, ffn_expansion_factor=2.6666, bias=False).to(device)
        self.combination_weight = nn.Sequential(
            nn.Conv2d(self.n_total_fts, n_graphs, kernel_size=1, stride=1, padding=0, bias=False),
            nn.Softmax(dim=1)).to(device)
        self.dc_estimator = DCestimator(12, 3, 12 * 2).to(device)
        self.ro00 = Parameter((torch.ones(n_graphs) * ro_init[0]).to(device))
        self.gamma00 = Parameter((torch.ones(n_graphs) * torch.log(gamma_init[0])).to(device))
        self.GTVmodule00 = GTVFast(nchannels_in, n_node_fts, n_graphs, connection_window, device, M_diag_init=1.0)
        self.muys00 = Parameter((torch.ones(n_graphs) * muy_init[0]).to(device))
        self.GLRmodule00 = GLRFast(nchannels_in, n_node_fts, n_graphs, connection_window, device, M_diag_init=1.0)

    def forward(self, patchs):
        if records_grad(self, patchs):
            # training: the solver and mixture run window_grad's HIP forward + HIP reverse;
            # the feature CNN / DC estimator / combination conv stay on PyTorch autograd
            feats = self.patchs_features_extraction(patchs)[0]
            graph_feats = feats[:, :-12]
            dc_term = self.dc_estimator(feats[:, -12:])
            x = WG.window_solve(self, patchs - dc_term, feats, with_taps=True)
            score = self.combination_weight(graph_feats)
            return WG.WinMixFn.apply(x, score.contiguous(), dc_term.contiguous())
        return self._forward_hip(patchs)

    @hip_forward
    def _forward_hip(self, patchs):
        feats = self.patchs_features_extraction(patchs)[0].contiguous()
        graph_feats = feats[:, :-12].contiguous()
        dc_term = self.dc_estimator(feats[:, -12:]).contiguous()
        y_tilde = (patchs - dc_term).contiguous()
        x = self.solve(y_tilde, graph_feats, feats)
        score = self.combination_weight(graph_feats).contiguous()
        return K.win_mix(x, score, dc_term)

    @torch.no_grad()
    def solve(self, y: torch.Tensor, graph_feats: torch.Tensor, feats: Optional[torch.Tensor] = None) -> torch.Tensor:
        """The unrolled ADMM / CG solver (REF7:936-1004) on y [B,Fs,H,W] -> x [B,G,Fs,H,W]."""
        g, f, fs = self.n_graphs, self.n_node_fts, y.shape[1]
        gtv, glr = self.GTVmodule00, self.GLRmodule00
        delta = gtv.edge_delta
        src = graph_feats if feats is None else feats
        wG, _ = K.win_edge_weights(src, 0, g, f, gtv.multiM.data.contiguous(), delta)
        wL, _ = K.win_edge_weights(src, 0, g, f, glr.multiM.data.contiguous(), delta)
        tG, tL = gtv.taps(), glr.taps()
        ro, mu, lg = self.ro00.data, self.muys00.data, self.gamma00.data
        alpha, beta = self.alphaCGD.data, self.betaCGD.data
        # the linear GTV passes (CG steps, first rhs) read pair weights (K loads per position
        # instead of K + K reverse-edge gathers); the prox rhs needs the raw directed weights
        pair = WIN_PAIR_WEIGHTS
        cG = K.win_pair_weights(wG, delta) if pair else wG

        def stages(rhs, ks):
            x, u = rhs, None
            for i, k in enumerate(ks):
                last = i == len(ks) - 1
                x, u = K.win_solver(0, x, rhs, cG, tG, ro, delta, g, fs, wL=wL, tapsL=tL, mu=mu, alpha=alpha[k],
                                    beta=beta[k] if u is not None else None, u_prev=u, want_u=not last, pair=pair)
            return x

        rhs, _ = K.win_solver(1, y, y, cG, tG, ro, delta, g, fs, pair=pair)              # REF7:945-949
        x = stages(rhs, [0, 1])                                                           # REF7:951-958
        rhs, _ = K.win_solver(2, x, y, wG, tG, ro, delta, g, fs, log_gamma=lg)            # REF7:960-967
        return stages(rhs, list(range(2, self.n_cgd_iters)))                              # REF7:970-990


class MultiScaleSequenceDenoiser(HipModule):
    """REF7:1019-1087: s0 y + s1 MixtureGTV(y), 24 graphs x 3 features on the 5x5 diamond (K=12)."""

    def __init__(self, device=None, n_cgd_iters: int = 4):
        super().__init__()
        self.device = device
        self.skip_connect_weight03 = Parameter(torch.tensor([0.1, 0.9], dtype=torch.float32, device=device))
        self.mixtureGLR_block03 = MixtureGTV(
            nchannels_in=3, n_graphs=24, n_node_fts=3, n_cnn_fts=128,
            connection_window=CONNECTION_FLAGS_5x5_small, n_cgd_iters=n_cgd_iters, alpha_init=0.5, beta_init=0.1,
            muy_init=torch.tensor([[0.1], [0.0], [0.0], [0.0]]), ro_init=torch.tensor([[0.1], [0.0], [0.0], [0.0]]),
            gamma_init=torch.tensor([[0.001], [0.0], [0.0], [0.0]]), device=device)

    def forward(self, patchs):
        return self.skip_connect_weight03[0] * patchs + self.skip_connect_weight03[1] * self.mixtureGLR_block03(patchs)
