"""Drop-in nn.Modules for the reference's graph-filter path, executed by libgrr.so.

Class names, constructor signatures, parameter names/shapes and therefore
``state_dict`` keys match the reference (REF = exploration/GGTV_GGLR_v1.0/
deep_multiscale_GGLR_GGTV_v1x0.py, REF13 = exploration/model_multiscale_mixture_GLR/
lib/model_GLR_GTV_deep_v13_no_latent.py), so reference checkpoints load unchanged.
The reference's plain-tensor constants (stats_kernel01..03, scaling_kernel01,
edge_delta, pad_dim_hw — REF:52-118, :613) become non-persistent buffers: they
follow ``.to()`` and stay out of the state_dict, as in the reference.

Forward passes of the graph filter run only through the HIP kernels (kernels.py);
GPU tensors are required.  When autograd records (training), every module here switches
to the differentiable path of solver_grad.py (HIP forward that keeps what the reverse
needs + hand-written HIP reverse kernels, each an opaque irdu:: op pair under torch.compile):
MixtureGTVGLR / LocalLowpassFilteringBlock (MIXTURE), GLRFast/GTVFast.forward and
extract_edge_weights (GRAPH_APPLY, EDGE_WEIGHTS), the module methods get_neighbors_pixels,
normalize_and_transform_features, stats_conv(_transpose), op_L_norm, op_C, op_C_transpose
(csrc/subapi_bwd.hip), LocalNonLinearBlock (LNB).  A HIP forward entered directly without a
reverse (``hip_forward``-wrapped internals) attaches a node whose backward raises, so
training can never silently skip gradients.
"""
from __future__ import annotations

import os
import warnings
from typing import List, Optional, Sequence

import torch
import torch.nn as nn
from torch.nn.parameter import Parameter

from . import kernels as K
from .compile_backend import HipModule
from . import ops as OPS
from . import solver_grad as SG

EDGE_DELTA = ((-1, 0), (0, -1), (0, 1), (1, 0))  # REF:42-53 (up, left, right, down)

# Inference: the half-resolution feature branch (2x2 conv, its LocalNonLinearBlocks, 1x1) runs on
# a second HIP stream beside the full-resolution branch (GRR_FEATURE_STREAMS=0: one stream)
FEATURE_STREAMS = os.environ.get("GRR_FEATURE_STREAMS", "1") == "1"
# Training: the same split for the forward and (by autograd's stream replay) the reverse of the branch
# (GRR_FEATURE_STREAMS_TRAIN=0: one stream).  Its earlier stalls came from library stream-K weight-gradient
# GEMMs co-resident on both streams; those reductions now run on grr_wgrad
FEATURE_STREAMS_TRAIN = os.environ.get("GRR_FEATURE_STREAMS_TRAIN", "1") == "1"
_SIDE_STREAMS = {}


def _side_stream(dev: torch.device) -> "torch.cuda.Stream":
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    if key not in _SIDE_STREAMS:
        _SIDE_STREAMS[key] = torch.cuda.Stream(device=dev)
    return _SIDE_STREAMS[key]


class _NoBackward(torch.autograd.Function):
    @staticmethod
    def forward(ctx, run, *tensors):
        out = run()
        return out if isinstance(out, torch.Tensor) else tuple(out)

    @staticmethod
    def backward(ctx, *grads):
        raise NotImplementedError("irdu_amd: HIP backward kernels are not built yet; "
                                  "run the graph filter under torch.no_grad()")


def records_grad(module: nn.Module, *tensors) -> bool:
    """True when autograd would record this call (training)."""
    return torch.is_grad_enabled() and (any(isinstance(t, torch.Tensor) and t.requires_grad for t in tensors)
                                        or any(p.requires_grad for p in module.parameters()))


# Chains of fused LocalNonLinearBlocks hand their intermediate tensors on in the channel-blocked layout
# (kernels.lnb_forward_c8: bitwise equal, fewer and wider memory instructions in each block).  Inference
# (eager and compiled: the irdu::lnb_forward_c8 op); training keeps [B, C, H, W].
BLOCKED_CHAINS = True
# The image filter's last feature 1x1 conv + the level's edge weights as one pass (kernels.feature_edges; v13
# feature CNN, F = 3, G <= 32, inference, eager and compiled).  Off: the two-pass path (conv1x1,
# edge_weights_block).
FUSED_FEATURE_EDGES = True


def run_blocks(blocks, x, first=None, out_blocked: bool = False):
    """x through the LocalNonLinearBlocks `blocks` in order; `first`, when given, replaces the first block's
    call (x -> its output, [B, C, H, W]).  Inference chains of fused blocks pass the blocked layout between
    the blocks.  Returns the output in [B, C, H, W]; with out_blocked, (output, is_blocked) where the last
    block may leave it blocked (for feature_edges)."""
    blocks = list(blocks)
    out = first(x) if first is not None else None
    rest = blocks[1:] if first is not None else blocks
    if out is None:
        out, rest = x, blocks
    b, c, h, w = out.shape
    chain = (BLOCKED_CHAINS and out.is_cuda and len(rest) >= (1 if out_blocked else 2)
             and all(isinstance(k, LocalNonLinearBlock) and k._blockable(h, w) and k.dim == c for k in rest)
             and not any(records_grad(k, out) for k in rest))
    if not chain:
        for k in rest:
            out = k(out)
        return (out, False) if out_blocked else out
    blocked = False
    for i, k in enumerate(rest):
        last = i == len(rest) - 1
        keep = not last or out_blocked
        out = k._forward_c8(out, blocked, keep)
        blocked = keep
    return (out, blocked) if out_blocked else out


def hip_forward(fn):
    """Run a HIP-backed forward; when autograd is recording, attach a node whose
    backward raises, so a training loop can never silently drop gradients."""
    def wrapper(self, *args, **kwargs):
        tensors = [a for a in args if isinstance(a, torch.Tensor)]
        if torch.is_grad_enabled() and (any(t.requires_grad for t in tensors)
                                        or any(p.requires_grad for p in self.parameters())):
            return _NoBackward.apply(lambda: fn(self, *args, **kwargs), *tensors, *self.parameters())
        return fn(self, *args, **kwargs)
    wrapper.__name__, wrapper.__doc__ = fn.__name__, fn.__doc__
    return wrapper


def _basis(c: int):
    z = torch.zeros(3, 3)
    k01 = z.clone(); k01[1, 1] = 1.0
    k02a = z.clone(); k02a[1, 1] = -1.0; k02a[1, 2] = 1.0
    k02b = z.clone(); k02b[1, 1] = -1.0; k02b[2, 1] = 1.0
    k03 = torch.tensor([[0.0, -1.0, 0.0], [-1.0, 4.0, -1.0], [0.0, -1.0, 0.0]])
    return [k.expand(c, 1, 3, 3).clone() for k in (k01, k02a, k02b, k03)]


class _GraphModule(HipModule):
    """Parameters shared by GLRFast and GTVFast (REF:14-125 / :243-356)."""

    def __init__(self, n_node_fts: int, n_graphs: int, M_diag_init: float = 0.4):
        super().__init__()
        self.n_channels = n_node_fts * n_graphs
        self.n_node_fts = n_node_fts
        self.n_graphs = n_graphs
        self.n_edges = len(EDGE_DELTA)
        self.buffer_size = self.n_edges
        c = self.n_channels
        self.register_buffer("edge_delta", torch.tensor(EDGE_DELTA, dtype=torch.int32), persistent=False)
        self.register_buffer("pad_dim_hw", torch.tensor([1, 1], dtype=torch.int32), persistent=False)
        b01, b02a, b02b, b03 = _basis(c)
        # parameters in the reference's registration order (state_dict order)
        self.stats_kernel_p01 = Parameter(torch.full((c, 1, 1, 1), 1.0))
        self.register_buffer("stats_kernel01", b01, persistent=False)
        self.stats_kernel_p02a = Parameter(torch.full((c, 1, 1, 1), 0.5))
        self.register_buffer("stats_kernel02a", b02a, persistent=False)
        self.stats_kernel_p02b = Parameter(torch.full((c, 1, 1, 1), 0.5))
        self.register_buffer("stats_kernel02b", b02b, persistent=False)
        self.stats_kernel_p03 = Parameter(torch.full((c, 1, 1, 1), 0.5))
        self.register_buffer("stats_kernel03", b03, persistent=False)
        self.multiM = Parameter(torch.full((n_graphs, n_node_fts), float(M_diag_init)))

    def extract_edge_weights(self, img_features: torch.Tensor):
        """[B,G,F,H,W] features -> (w [B,G,4,H,W], degree [B,G,H,W]) (REF:160-175)."""
        if records_grad(self, img_features):
            return SG.edge_weights(self, img_features)
        return self._edge_weights(img_features)

    @torch.no_grad()
    def _edge_weights(self, img_features: torch.Tensor):
        b, g, f, h, w = img_features.shape
        x = img_features.reshape(b, g * f, h, w).contiguous()
        return OPS.edge_weights(x, 0, g, f, self.multiM, with_degree=True)

    def neighbor_table(self, h: int, w: int) -> torch.Tensor:
        """int32 [4,H,W] flat indices of the neighbours each edge reads (REF:128-144)."""
        return K.neighbor_table(h, w, self.multiM.device)

    # -- the reference's module methods, standalone (the solver fuses them; csrc/subapi_ops.hip) --
    # Differentiable like the reference's ATen compositions: under autograd they run the same HIP
    # forwards with their reverses (csrc/subapi_bwd.hip) through solver_grad's opaque functions.
    def _stencil_params(self):
        return (self.stats_kernel_p01, self.stats_kernel_p02a, self.stats_kernel_p02b, self.stats_kernel_p03)

    def get_neighbors_pixels(self, img_features):
        """[B,C,H,W] -> [B,C,4,H,W]: the replicate-clamped up/left/right/down neighbours (REF:128-144)."""
        if records_grad(self, img_features):
            return SG.NEIGHBORS([], img_features.contiguous())
        return OPS.neighbor_gather(img_features.contiguous())

    def normalize_and_transform_features(self, img_features):
        """[B,G,F,H,W] -> [B,G*F,H,W]: L2-normalised over F (eps 1e-12), scaled by multiM (REF:146-157)."""
        if records_grad(self, img_features):
            return SG.NORMALIZE([], img_features.contiguous(), self.multiM)
        return OPS.normalize_features(img_features.contiguous(), self.multiM)

    def stats_conv(self, patchs):
        """S x, depthwise 3x3 cross stencil with a replicate frame (REF:177-195)."""
        if records_grad(self, patchs):
            return SG.STATS_CONV([0], patchs.contiguous(), *self._stencil_params())
        return OPS.stats_conv(patchs.contiguous(), self, False)

    def stats_conv_transpose(self, patchs):
        """S^T x, conv_transpose2d(padding=1) of the same stencil, zero frame (REF:197-215)."""
        if records_grad(self, patchs):
            return SG.STATS_CONV([1], patchs.contiguous(), *self._stencil_params())
        return OPS.stats_conv(patchs.contiguous(), self, True)


class GLRFast(_GraphModule):
    """Graph-Laplacian regulariser S^T (I - W) S (REF:13-237)."""

    def forward(self, patchs, edge_weights, node_degree=None):
        if records_grad(self, patchs, edge_weights):
            return SG.graph_apply(self, "glr", patchs, edge_weights)
        return self._hip_apply(patchs, edge_weights)

    def op_L_norm(self, img_signals, edge_weights, node_degree=None):
        """x - sum_e w_e x(clamp(p + delta_e)) (REF:218-228); x [B,G,F,H,W], w [B,G,4,H,W]."""
        if records_grad(self, img_signals, edge_weights):
            return SG.OP_L_NORM([], img_signals.contiguous(), edge_weights.contiguous())
        return OPS.glr_op_L_norm(img_signals.contiguous(), edge_weights.contiguous())

    @torch.no_grad()
    def _hip_apply(self, patchs, edge_weights):
        b, g, f, h, w = patchs.shape
        out = OPS.system_half(patchs.reshape(b, g * f, h, w).contiguous(), edge_weights.contiguous(), None,
                              self, None, None, None, g)
        return out.view(b, g, f, h, w)


class GTVFast(_GraphModule):
    """Graph total variation C^T C with C = W (S - S shifted) (REF:242-523)."""

    def forward(self, patchs, edge_weights, node_degree=None):
        if records_grad(self, patchs, edge_weights):
            return SG.graph_apply(self, "gtv", patchs, edge_weights)
        return self._hip_apply(patchs, edge_weights)

    def op_C(self, img_signals, edge_weights, node_degree=None):
        """Edge signals E_e = w_e (S x - (S x)(clamp(p + delta_e))), [B,G,F,4,H,W] (REF:452-467)."""
        if records_grad(self, img_signals, edge_weights):
            return SG.OP_C([], img_signals.contiguous(), edge_weights.contiguous(), *self._stencil_params())
        return OPS.gtv_op_C(img_signals.contiguous(), edge_weights.contiguous(), self)

    def op_C_transpose(self, edge_signals, edge_weights, node_degree=None):
        """S^T of the frame-dropped scatter of w_e E_e (REF:469-516) -> [B,G,F,H,W]."""
        if records_grad(self, edge_signals, edge_weights):
            return SG.OP_C_T([], edge_signals.contiguous(), edge_weights.contiguous(), *self._stencil_params())
        return OPS.gtv_op_C_transpose(edge_signals.contiguous(), edge_weights.contiguous(), self)

    @torch.no_grad()
    def _hip_apply(self, patchs, edge_weights):
        b, g, f, h, w = patchs.shape
        c = OPS.gtv_pair_weights(edge_weights.contiguous())
        out = OPS.system_half(patchs.reshape(b, g * f, h, w).contiguous(), None, c, None, self, None, None, g)
        return out.view(b, g, f, h, w)


# ---------------------------------------------------------------------------
# Feature CNN building blocks (REF:911-964; REF13:541-575)
# ---------------------------------------------------------------------------
class CustomLayerNorm(HipModule):
    def __init__(self, nchannels, nsubnets):
        super().__init__()
        self.nsubnets = nsubnets
        self.nchannels = nchannels
        self.weighted_transform = nn.Conv2d(nchannels, nchannels, kernel_size=1, stride=1, groups=nchannels,
                                            bias=False)

    def forward(self, x):  # stock PyTorch (encoder/decoder use; hot path goes through LocalNonLinearBlock)
        b, c, h, w = x.shape
        xs = x.reshape(b, self.nsubnets, c // self.nsubnets, h, w)
        xs = xs / torch.sqrt(xs.var(dim=2, keepdim=True, correction=1) + 1e-5)
        return self.weighted_transform(xs.reshape(b, c, h, w))


class LocalGatedLinearBlock(HipModule):
    def __init__(self, dim, hidden_dim, nsubnets):
        super().__init__()
        self.channels_linear_op = nn.Conv2d(dim, hidden_dim * 2, kernel_size=1, bias=False, groups=nsubnets)
        self.channels_local_linear_op = nn.Conv2d(hidden_dim * 2, hidden_dim * 2, kernel_size=3, stride=1, padding=1,
                                                  padding_mode="replicate", groups=hidden_dim * 2, bias=False)
        self.project_out = nn.Conv2d(hidden_dim, dim, kernel_size=1, bias=False, groups=nsubnets)

    def forward(self, x):
        x = self.channels_linear_op(x)
        mask, x = self.channels_local_linear_op(x).chunk(2, dim=1)
        return self.project_out(torch.sigmoid(mask) * mask * x)


class LocalNonLinearBlock(HipModule):
    """skip0 * x + skip1 * GatedLinear(LayerNorm(x)).  nsubnets == 1 runs the fused HIP block."""

    def __init__(self, dim, hidden_dim, nsubnets):
        super().__init__()
        self.dim, self.hidden_dim, self.nsubnets = dim, hidden_dim, nsubnets
        self.norm = CustomLayerNorm(dim, nsubnets)
        self.local_linear = LocalGatedLinearBlock(dim, hidden_dim, nsubnets)
        self.skip_weight = Parameter(torch.tensor([1.0, 1.0], dtype=torch.float32))

    def forward(self, x):
        if self.nsubnets != 1:
            # grouped variant (encoder/decoder configs only, outside the hot path): stock PyTorch-ROCm ops
            return self.skip_weight[0] * x + self.skip_weight[1] * self.local_linear(self.norm(x))
        if records_grad(self, x):
            ll = self.local_linear
            return SG.LNBFn.apply(x.contiguous(), self.norm.weighted_transform.weight, ll.channels_linear_op.weight,
                                  ll.channels_local_linear_op.weight, ll.project_out.weight, self.skip_weight)
        return self._forward_hip(x)

    @torch.no_grad()
    def forward_replicated(self, src, x=None):
        """Inference forward when the block input is copies of src along channels (C <= 128):
        GEMM1 on src; x (the materialised copies) may be None, the skip then reads src."""
        ll = self.local_linear
        c, hid = self.dim, self.hidden_dim
        if c > 128 or self.nsubnets != 1:
            if x is None:
                x = OPS.repeat_graphs(src, c // src.shape[1])
            return self._forward_hip(x)
        return OPS.lnb_forward_rep(src, x, self.norm.weighted_transform.weight.view(c),
                                   ll.channels_linear_op.weight.view(2 * hid, c),
                                   ll.channels_local_linear_op.weight.view(2 * hid, 9),
                                   ll.project_out.weight.view(c, hid), self.skip_weight)

    def _blockable(self, h: int, w: int) -> bool:
        return self.nsubnets == 1 and K.lnb_c8_ok(self.dim, self.hidden_dim, h, w)

    def _forward_c8(self, x, in_c8: bool, out_c8: bool):
        """Inference forward with x / out in the channel-blocked layout (kernels.lnb_forward_c8)."""
        ll = self.local_linear
        c, hid = self.dim, self.hidden_dim
        return OPS.lnb_forward_c8(x, c, self.norm.weighted_transform.weight.view(c),
                                ll.channels_linear_op.weight.view(2 * hid, c),
                                ll.channels_local_linear_op.weight.view(2 * hid, 9),
                                ll.project_out.weight.view(c, hid), self.skip_weight, in_c8, out_c8)

    @hip_forward
    def _forward_hip(self, x):
        ll = self.local_linear
        c, hid = self.dim, self.hidden_dim
        return OPS.lnb_forward(x.contiguous(), self.norm.weighted_transform.weight.view(c),
                               ll.channels_linear_op.weight.view(2 * hid, c),
                               ll.channels_local_linear_op.weight.view(2 * hid, 9),
                               ll.project_out.weight.view(c, hid), self.skip_weight)


# ---------------------------------------------------------------------------
# The solver block
# ---------------------------------------------------------------------------
class MixtureGTVGLR(HipModule):
    """Two-scale GGTV+GGLR unrolled solver (REF:526-811).

    ``n_cgd_iters`` (default 3 = the reference) sets the number S of unrolled
    stages; S > 3 follows the reference's extension pattern (REF:797-807).
    ``feature_extractor``: "v1" = the v1.0 1x1 / 2x2 convs (REF:556-612);
    "v13" = the image-domain 3x LocalNonLinearBlock CNN of REF13:612-698.
    """

    def __init__(self, n_graphs, n_node_fts, alpha_init, beta_init, muy_init, ro_init, gamma_init,
                 n_cgd_iters: int = 3, feature_extractor: str = "v1"):
        super().__init__()
        self.n_graphs = n_graphs
        self.n_node_fts = n_node_fts
        self.n_channels = c = n_graphs * n_node_fts
        self.n_cgd_iters = n_cgd_iters
        self.feature_extractor = feature_extractor
        muy_init, ro_init, gamma_init = (torch.as_tensor(v, dtype=torch.float32) for v in (muy_init, ro_init, gamma_init))
        self.alphaCGD = Parameter(torch.ones((n_cgd_iters, n_graphs)) * alpha_init)
        self.betaCGD = Parameter(torch.ones((n_cgd_iters, n_graphs)) * beta_init)
        if feature_extractor == "v1":
            self.patchs_features_extraction00 = nn.Sequential(nn.Conv2d(c, 2 * c, 1, bias=False))
        else:
            hid = int(c * 8 / 3)
            self.patchs_features_extraction00 = nn.Sequential(
                *[LocalNonLinearBlock(c, hid, 1) for _ in range(3)], nn.Conv2d(c, 2 * c, 1, bias=False))
        self.ro00 = Parameter(torch.ones(n_graphs) * torch.log(ro_init[0]))
        self.gamma00 = Parameter(torch.ones(n_graphs) * torch.log(gamma_init[0]))
        self.GTVmodule00 = GTVFast(n_node_fts, n_graphs, M_diag_init=1.0)
        self.muys00 = Parameter(torch.ones(n_graphs) * torch.log(muy_init[0]))
        self.GLRmodule00 = GLRFast(n_node_fts, n_graphs, M_diag_init=1.0)
        if feature_extractor == "v1":
            self.patchs_features_extraction01 = nn.Sequential(nn.Conv2d(c, c, 2, stride=2, bias=False),
                                                              nn.Conv2d(c, 2 * c, 1, bias=False))
        else:
            hid = int(c * 8 / 3)
            self.patchs_features_extraction01 = nn.Sequential(
                nn.Conv2d(c, c, 2, stride=2, bias=False), *[LocalNonLinearBlock(c, hid, 1) for _ in range(3)],
                nn.Conv2d(c, 2 * c, 1, bias=False))
        self.register_buffer("scaling_kernel01", torch.full((c, 1, 2, 2), 0.25), persistent=False)
        self.ro01 = Parameter(torch.ones(n_graphs) * torch.log(ro_init[1]))
        self.gamma01 = Parameter(torch.ones(n_graphs) * torch.log(gamma_init[1]))
        self.GTVmodule01 = GTVFast(n_node_fts, n_graphs, M_diag_init=1.0)
        self.muys01 = Parameter(torch.ones(n_graphs) * torch.log(muy_init[1]))
        self.GLRmodule01 = GLRFast(n_node_fts, n_graphs, M_diag_init=1.0)

    # -- feature maps (a13) --------------------------------------------------
    @staticmethod
    def _down(y: torch.Tensor, weight: torch.Tensor, src: Optional[torch.Tensor]) -> torch.Tensor:
        """2x2/s2 conv of y.  When y is src replicated over the graphs (MultiScaleGraphFilter),
        the conv of the replicas equals the conv of src with the weights summed over the
        replicas: K = 4 Cin instead of 4 G Cin (same value up to fp32 summation order)."""
        if src is None:
            return OPS.conv2x2s2(y, weight)
        return OPS.conv2x2s2(src, weight, fold=True)

    def features(self, y: torch.Tensor, src: Optional[torch.Tensor] = None, half_tail=None, project: bool = True):
        """f0, f1 (a13).  half_tail(f1), when given, runs right after the half-resolution branch on
        the same stream and its tuple of tensors is returned in place of f1.  project=False (v13, inference):
        each branch stops before its last 1x1 conv and yields (x, is_blocked), the last block's output for
        feature_edges."""
        s0, s1 = self.patchs_features_extraction00, self.patchs_features_extraction01
        if self.feature_extractor == "v1":
            f0 = OPS.conv1x1(y, s0[0].weight)
            f1 = OPS.conv1x1(self._down(y, s1[0].weight, src), s1[1].weight)
            return f0, (half_tail(f1) if half_tail is not None else f1)
        ref = y if y is not None else src

        def half():
            if project:
                f1 = OPS.conv1x1(run_blocks(list(s1)[1:4], self._down(y, s1[0].weight, src)), s1[4].weight)
            else:
                f1 = run_blocks(list(s1)[1:4], self._down(y, s1[0].weight, src), out_blocked=True)
            return half_tail(f1) if half_tail is not None else f1

        side = None
        if FEATURE_STREAMS and ref.is_cuda and not torch.compiler.is_compiling() \
                and not torch.cuda.is_current_stream_capturing():
            main = torch.cuda.current_stream(ref.device)
            side = _side_stream(ref.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                f1 = half()
        else:
            f1 = half()
        blocks = list(s0)[:3]
        # the first block's input replicates src over the graphs: its GEMM1 runs on src (K = F)
        first = (lambda _y: blocks[0].forward_replicated(src, _y)) if src is not None else None
        if project:
            f0 = OPS.conv1x1(run_blocks(blocks, y, first=first), s0[3].weight)
        else:
            f0 = run_blocks(blocks, y, first=first, out_blocked=True)
        if side is not None:
            main.wait_stream(side)
            for t in (f1 if isinstance(f1, tuple) else (f1,)):
                if isinstance(t, torch.Tensor):
                    t.record_stream(main)
        return f0, f1

    def features_train(self, y: torch.Tensor):
        """Differentiable feature maps (training): HIP convs with autograd reverses."""
        s0, s1 = self.patchs_features_extraction00, self.patchs_features_extraction01
        if self.feature_extractor == "v1":
            f0 = SG.Conv1x1Fn.apply(y, s0[0].weight)
            f1 = SG.Conv1x1Fn.apply(SG.Conv2x2s2Fn.apply(y, s1[0].weight), s1[1].weight)
            return f0, f1
        def half():
            f1 = SG.Conv2x2s2Fn.apply(y, s1[0].weight)
            for blk in list(s1)[1:4]:
                f1 = blk(f1)
            return SG.Conv1x1Fn.apply(f1.contiguous(), s1[4].weight)

        # the half-resolution branch on the side stream (its reverse then also runs there: autograd
        # replays a node on the stream its forward ran on).  Cross-stream memory: y (main) is read by
        # side kernels in both directions and f1 (side) by the main-stream solver, so each is
        # recorded on the other stream -- the caching allocator then cannot hand either block to a
        # new tensor while the other stream may still read it.
        side = None
        if FEATURE_STREAMS_TRAIN and y.is_cuda and not torch.compiler.is_compiling() \
                and not torch.cuda.is_current_stream_capturing():
            main = torch.cuda.current_stream(y.device)
            side = _side_stream(y.device)
            side.wait_stream(main)
            y.record_stream(side)
            with torch.cuda.stream(side):
                f1 = half()
        else:
            f1 = half()
        f0 = y
        for blk in list(s0)[:3]:
            f0 = blk(f0)
        f0 = SG.Conv1x1Fn.apply(f0.contiguous(), s0[3].weight)
        if side is not None:
            main.wait_stream(side)
            f1.record_stream(main)
        return f0, f1

    # -- solver (a3-a17) -----------------------------------------------------
    def _solve(self, y: Optional[torch.Tensor], skip: Optional[torch.Tensor] = None,
               src: Optional[torch.Tensor] = None) -> torch.Tensor:
        """src: optional [B, F, H, W] image that y replicates over the G graphs (y[:, gF + i] =
        src[:, i]); lets the replicated-input steps run on src.  With src, y may be None: the
        replicated input is then never materialised (first feature block, 2x2 conv and both
        right-hand sides read src; REF13:918-921)."""
        g, f = self.n_graphs, self.n_node_fts
        if y is None:
            if src is None:
                raise ValueError("MixtureGTVGLR: need y or src")
            if self.feature_extractor != "v13" or skip is not None:   # those paths read y itself
                y = OPS.repeat_graphs(src, g)
        ref = y if y is not None else src
        b, c, h, w = ref.shape
        if y is not None and c != self.n_channels:
            raise ValueError(f"MixtureGTVGLR: expected {self.n_channels} channels, got {c}")
        if h % 2 or w % 2:
            raise ValueError(f"MixtureGTVGLR: H, W must be even for the 2x2 scale (got {h}x{w})")
        if src is not None and (src.shape[1] != f or src.shape[0] != b or tuple(src.shape[2:]) != (h, w)):
            raise ValueError("MixtureGTVGLR: src must be [B, F, H, W]")
        G0, L0, G1, L1 = self.GTVmodule00, self.GLRmodule00, self.GTVmodule01, self.GLRmodule01

        # the last 1x1 conv of each feature branch and the level's edge weights in one pass (v13, eager)
        fuse = (FUSED_FEATURE_EDGES and self.feature_extractor == "v13" and ref.is_cuda
                and K.feature_edges_ok(g * f, g, f, h, w) and K.feature_edges_ok(g * f, g, f, h // 2, w // 2))
        s0, s1 = self.patchs_features_extraction00, self.patchs_features_extraction01

        def half_tail(f1):
            # the half level's edge weights and its part of rhs A (ro1 G1 D y, REF:738-749)
            if fuse:
                wG1, cG1, wL1 = OPS.feature_edges(f1[0], f1[1], s1[4].weight, g, f, G1.multiM, L1.multiM)
            else:
                wG1, cG1, wL1 = OPS.edge_weights_block(f1, g, f, G1.multiM, L1.multiM)
            yd = OPS.pool2(y) if src is None else OPS.repeat_graphs(OPS.pool2(src), g)   # D y
            return wG1, cG1, wL1, OPS.gtv_rhs_half(yd, cG1, G1, False, None, g)

        f0, (wG1, cG1, wL1, t) = self.features(y, src, half_tail, project=not fuse)
        if fuse:
            wG0, cG0, wL0 = OPS.feature_edges(f0[0], f0[1], s0[3].weight, g, f, G0.multiM, L0.multiM)
        else:
            wG0, cG0, wL0 = OPS.edge_weights_block(f0, g, f, G0.multiM, L0.multiM)
        del f0
        mu0, mu1, ro0, ro1 = self.muys00, self.muys01, self.ro00, self.ro01
        alpha, beta = self.alphaCGD, self.betaCGD
        n_st = alpha.shape[0]

        # rhs A: b_A = y + ro0 G0 y + ro1 U(G1 D y)                     (REF:738-749)
        if y is None:
            b_a, xd = OPS.gtv_rhs_full(src, True, src, True, cG0, G0, False, None, ro0, t, ro1, g, want_pool=True)
        else:
            b_a, xd = OPS.gtv_rhs_full(y, False, y, False, cG0, G0, False, None, ro0, t, ro1, g, want_pool=True)
        u, u_spare = None, None
        if n_st >= 3 and OPS.first_pair_supported(b_a, g):
            # stage 0, the prox rhs B and stage 1 in one pass: x1, D x1, t0, t1 and both prox terms stay on
            # chip (REF:751-790 at k = 0, 1); the pairs below then end on stage S-1 with its skip
            b_b, x, u, xd = OPS.system_first_pair(b_a, xd, src if y is None else y, y is None, wL0, cG0, wG0, L0, G0,
                                                  mu0, ro0, self.gamma00, wL1, cG1, wG1, L1, G1, mu1, ro1,
                                                  self.gamma01, alpha[0], alpha[1], g)
            del b_a, wG0, wG1
            pair = OPS.step2_supported(x, g)
            k = 2
        else:
            # stage 0: x1 = b_A + alpha0 (b_A - A b_A)                     (REF:751-753)
            last = n_st == 1
            t = OPS.system_half(xd, wL1, cG1, L1, G1, mu1, ro1, g)
            x, _, xd = OPS.system_step(b_a, b_a, None, t, wL0, cG0, L0, G0, mu0, ro0, alpha[0], None, g,
                                       want_u=False, want_pool=not last, skip=skip if last else None,
                                       y_skip=y if last else None)
            del b_a
            if last:
                return x
            # GTV proximal step -> rhs B                                   (REF:757-781)
            t = OPS.gtv_rhs_half(xd, wG1, G1, True, self.gamma01, g)
            if y is None:
                b_b, _ = OPS.gtv_rhs_full(x, False, src, True, wG0, G0, True, self.gamma00, ro0, t, ro1, g)
            else:
                b_b, _ = OPS.gtv_rhs_full(x, False, y, False, wG0, G0, True, self.gamma00, ro0, t, ro1, g)
            del wG0, wG1
            pair = OPS.step2_supported(x, g)
            k = 1
        while k < n_st:                                              # (REF:784-790, :797-807)
            if pair and k + 1 < n_st:
                # stages k, k+1 in one pass, both half levels inside: t_k, x_{k+1}, u_{k+1},
                # t_{k+1} stay on chip
                last = k + 1 == n_st - 1
                x, u_new, xd = OPS.system_step2(x, b_b, u, xd, wL0, cG0, L0, G0, mu0, ro0, wL1, cG1, L1, G1, mu1,
                                                ro1, alpha[k], beta[k] if k >= 2 else None, alpha[k + 1], beta[k + 1],
                                                g, want_u=not last, want_pool=not last, skip=skip if last else None,
                                                y_skip=y if last else None, u_out=u_spare)
                u_spare, u = u, u_new
                k += 2
                continue
            last = k == n_st - 1
            t = OPS.system_half(xd, wL1, cG1, L1, G1, mu1, ro1, g)
            x, u, xd = OPS.system_step(x, b_b, u, t, wL0, cG0, L0, G0, mu0, ro0, alpha[k],
                                       beta[k] if k >= 2 else None, g, want_u=not last, want_pool=not last,
                                       skip=skip if last else None, y_skip=y if last else None, u_out=u)
            k += 1
        return x

    def forward(self, patchs: torch.Tensor, _skip: Optional[torch.Tensor] = None,
                _src: Optional[torch.Tensor] = None) -> torch.Tensor:
        if records_grad(self, patchs, _skip):
            y = patchs.contiguous()
            b, c, h, w = y.shape
            if c != self.n_channels or h % 2 or w % 2:
                raise ValueError(f"MixtureGTVGLR: expected [B,{self.n_channels},H,W] with even H, W, "
                                 f"got {tuple(y.shape)}")
            f0, f1 = self.features_train(y)
            x = SG.mixture_solve(self, y, f0, f1)
            return x if _skip is None else _skip[0] * y + _skip[1] * x
        with torch.no_grad():
            return self._solve(patchs.contiguous(), _skip, None if _src is None else _src.contiguous())


class LocalLowpassFilteringBlock(HipModule):
    """skip0 * x + skip1 * MixtureGTVGLR(x), the skip fused into the last stage (REF:967-988)."""

    def __init__(self, dim, nsubnets, ngraphs, n_cgd_iters: int = 3):
        super().__init__()
        self.local_filter = MixtureGTVGLR(
            n_graphs=ngraphs, n_node_fts=dim // ngraphs, alpha_init=0.5, beta_init=0.1,
            muy_init=torch.tensor([[0.001], [0.0001]]), ro_init=torch.tensor([[0.0001], [0.0001]]),
            gamma_init=torch.tensor([[0.0001], [0.0001]]), n_cgd_iters=n_cgd_iters)
        self.skip_weight = Parameter(torch.tensor([0.5, 0.5], dtype=torch.float32))

    def forward(self, x):
        if records_grad(self, x):
            return self.local_filter(x, _skip=self.skip_weight)
        return self.local_filter(x, _skip=self.skip_weight.detach())


class MultiScaleGraphFilter(HipModule):
    """Image-domain GGTV-GGLR filter (REF13:887-926): RGB replicated over G graphs,
    MixtureGTVGLR with the v13 feature CNN, then a 1x1 projection to the output."""

    def __init__(self, n_channels_in=3, n_channels_out=3, ngraphs=16, n_cgd_iters: int = 3):
        super().__init__()
        self.ngraphs = ngraphs
        self.n_channels_in = n_channels_in
        self.localfilter = MixtureGTVGLR(
            n_graphs=ngraphs, n_node_fts=n_channels_in, alpha_init=0.5, beta_init=0.1,
            muy_init=torch.tensor([[0.001], [0.0001]]), ro_init=torch.tensor([[0.0001], [0.0001]]),
            gamma_init=torch.tensor([[0.0001], [0.0001]]), n_cgd_iters=n_cgd_iters, feature_extractor="v13")
        self.linear_combination = nn.Conv2d(ngraphs * n_channels_in, n_channels_out, 1, bias=False)

    def forward(self, img):
        img = img.contiguous()
        if records_grad(self, img):
            y = self.localfilter(SG.RepeatGraphsFn.apply(img, self.ngraphs))
            return SG.Conv1x1Fn.apply(y.contiguous(), self.linear_combination.weight)
        return self._forward_inference(img)

    @torch.no_grad()
    def _forward_inference(self, img):
        # the G-fold replicated input (REF13:918-921) is never materialised: the solver reads img
        y = self.localfilter._solve(None, None, img)
        return OPS.conv1x1(y, self.linear_combination.weight)


# ---------------------------------------------------------------------------
# v1.0 end-to-end model (REF:991-1174).  Encoder/decoder are outside the hot path:
# their convolutions run as stock PyTorch-ROCm ops; LocalNonLinearBlocks with
# nsubnets == 1 and the four filter blocks run on the HIP kernels.
# ---------------------------------------------------------------------------
class ReginalPixelEmbeding(HipModule):
    def __init__(self, n_channels_in=3, dim=48, bias=False):
        super().__init__()
        self.channels_local_linear_op01 = nn.Conv2d(n_channels_in, dim, kernel_size=3, stride=1, padding=1,
                                                    padding_mode="replicate", bias=False)

    def forward(self, x):
        return self.channels_local_linear_op01(x)


class Downsampling(HipModule):
    def __init__(self, dim_in, dim_out, nsubnets):
        super().__init__()
        self.local_linear = nn.Conv2d(dim_in, dim_out, kernel_size=2, stride=2, padding=0, groups=nsubnets, bias=False)

    def forward(self, x):
        return self.local_linear(x)


class Upsampling(HipModule):
    def __init__(self, dim_in, dim_out, nsubnets):
        super().__init__()
        self.local_linear = nn.ConvTranspose2d(dim_in, dim_out, kernel_size=2, stride=2, padding=0, groups=nsubnets,
                                               bias=False)

    def forward(self, x):
        return self.local_linear(x)


_MIOPEN_CHECKED = False


def _warn_miopen_find_db() -> None:
    """Once per process: a drop-in training script that never called irdu_amd.miopen_training_defaults()
    (and does not set MIOPEN_DEBUG_DISABLE_FIND_DB itself) trains the v1.0 model's stock convolutions
    with MIOpen's user find-db, 2.7-4.0 s per C4 step instead of 1.03 s after a box's first run
    (DESIGN.md §4.r4).  Importing the package changes no process-wide setting, so this only warns."""
    global _MIOPEN_CHECKED
    if _MIOPEN_CHECKED or torch.compiler.is_compiling():
        return
    _MIOPEN_CHECKED = True
    if "MIOPEN_DEBUG_DISABLE_FIND_DB" not in os.environ:
        warnings.warn("irdu_amd: training AbtractMultiScaleGraphFilter without MIOPEN_DEBUG_DISABLE_FIND_DB set; "
                      "call irdu_amd.miopen_training_defaults() before the first convolution (MIOpen's find-db "
                      "costs seconds of host time per step on later runs, DESIGN.md §4.r4)", RuntimeWarning,
                      stacklevel=3)


class AbtractMultiScaleGraphFilter(HipModule):
    def __init__(self, n_channels_in=3, n_channels_out=3, dims=(48, 64, 96, 128), hidden_dims=(128, 192, 256, 384),
                 nsubnets=(1, 1, 1, 1), ngraphs=(4, 4, 8, 8), num_blocks=(4, 6, 6, 8), num_blocks_out=4,
                 n_cgd_iters: int = 3):
        super().__init__()
        dims, hidden_dims, nsubnets, ngraphs, num_blocks = map(list, (dims, hidden_dims, nsubnets, ngraphs, num_blocks))

        def blocks(i, n):
            return nn.Sequential(*[LocalNonLinearBlock(dims[i], hidden_dims[i], nsubnets[i]) for _ in range(n)])

        self.patch_3x3_embeding = ReginalPixelEmbeding(n_channels_in, dims[0])
        self.encoder_scale_00 = blocks(0, num_blocks[0])
        self.down_sample_00_01 = Downsampling(dims[0], dims[1], nsubnets[0])
        self.encoder_scale_01 = blocks(1, num_blocks[1])
        self.down_sample_01_02 = Downsampling(dims[1], dims[2], nsubnets[1])
        self.encoder_scale_02 = blocks(2, num_blocks[2])
        self.down_sample_02_03 = Downsampling(dims[2], dims[3], nsubnets[2])
        self.encoder_scale_03 = blocks(3, num_blocks[3])
        self.localfilter_scale_00 = LocalLowpassFilteringBlock(dims[0], nsubnets[0], ngraphs[0], n_cgd_iters)
        self.localfilter_scale_01 = LocalLowpassFilteringBlock(dims[1], nsubnets[1], ngraphs[1], n_cgd_iters)
        self.localfilter_scale_02 = LocalLowpassFilteringBlock(dims[2], nsubnets[2], ngraphs[2], n_cgd_iters)
        self.localfilter_scale_03 = LocalLowpassFilteringBlock(dims[3], nsubnets[3], ngraphs[3], n_cgd_iters)
        self.up_sample_03_02 = Upsampling(dims[3], dims[2], nsubnets[3])
        self.combine_channels_02 = nn.Conv2d(dims[2] * 2, dims[2], kernel_size=1, bias=False, groups=nsubnets[2])
        self.decoder_scale_02 = blocks(2, num_blocks[2])
        self.up_sample_02_01 = Upsampling(dims[2], dims[1], nsubnets[2])
        self.combine_channels_01 = nn.Conv2d(dims[1] * 2, dims[1], kernel_size=1, bias=False, groups=nsubnets[1])
        self.decoder_scale_01 = blocks(1, num_blocks[1])
        self.up_sample_01_00 = Upsampling(dims[1], dims[0], nsubnets[1])
        self.combine_channels_00 = nn.Conv2d(dims[0] * 2, dims[0], kernel_size=1, bias=False, groups=nsubnets[0])
        self.decoder_scale_00 = blocks(0, num_blocks[0])
        self.refining_block = blocks(0, num_blocks_out)
        self.linear_output = nn.Conv2d(dims[0], n_channels_out, kernel_size=1, bias=False)

    def encode(self, img):
        e0 = self.encoder_scale_00(self.patch_3x3_embeding(img))
        e1 = self.encoder_scale_01(self.down_sample_00_01(e0))
        e2 = self.encoder_scale_02(self.down_sample_01_02(e1))
        e3 = self.encoder_scale_03(self.down_sample_02_03(e2))
        return e0, e1, e2, e3

    def filtering(self, coefs):
        e0, e1, e2, e3 = coefs
        return (self.localfilter_scale_00(e0), self.localfilter_scale_01(e1),
                self.localfilter_scale_02(e2), self.localfilter_scale_03(e3))

    def decode(self, coefs):
        e0, e1, e2, e3 = coefs
        d = self.combine_channels_02(torch.cat([self.up_sample_03_02(e3), e2], 1))
        d = self.decoder_scale_02(d)
        d = self.combine_channels_01(torch.cat([self.up_sample_02_01(d), e1], 1))
        d = self.decoder_scale_01(d)
        d = self.combine_channels_00(torch.cat([self.up_sample_01_00(d), e0], 1))
        d = self.decoder_scale_00(d)
        return self.linear_output(self.refining_block(d))

    def enc_dec(self, img):
        return self.decode(self.encode(img))

    def forward(self, img):
        if self.training and torch.is_grad_enabled():
            _warn_miopen_find_db()
        return self.decode(self.filtering(self.encode(img)))
