"""Training-path autograd functions that stay opaque under ``torch.compile``.

The reference trains the compiled model (``model.compile()`` then the loop of
scripts_v2/run_abtract_lightformer_GGTV_GGLR_sigma25.py:130, :186-207).  Each differentiable HIP
operation of the training path (solver_grad.py) is written as a pair of pure functions

    fwd(consts, *inputs)                    -> (outputs, saved)   saved: extra tensors the reverse needs
    bwd(consts, inputs, outs, saved, gouts, needs) -> one gradient (or None) per input

and wrapped by :class:`OpaqueFunction` in two forms:

* eager: a ``torch.autograd.Function`` (no dispatcher hop per launch);
* while Dynamo traces (``torch.compiler.is_compiling()``): two ``torch.library`` custom ops,
  ``irdu::<name>`` (outputs + saved tensors) and ``irdu::<name>_backward`` (input gradients),
  linked by ``register_autograd``.  Dynamo and AOTAutograd see one opaque node per direction with
  fake kernels giving the shapes, so the HIP launches never enter Inductor (no Triton) and the
  compiled step runs exactly the kernels of the eager step.

``FORCE_OPS`` routes eager calls through the custom ops as well (tests capture the joint
forward/backward graph with fake tensors on CPU).
"""
from typing import Callable, List, Sequence

import torch
from torch import Tensor

NS = "irdu"
FORCE_OPS = False
OPAQUE = {}


class OpaqueFunction:
    def __init__(self, name: str, n_out: int, fwd: Callable, bwd: Callable, fake: Callable):
        self.name, self.n_out = name, n_out
        self.fwd, self.bwd, self.fake = fwd, bwd, fake
        spec = self

        class _Eager(torch.autograd.Function):
            @staticmethod
            def forward(ctx, consts, *inputs):
                outs, saved = spec.fwd(list(consts), *inputs)
                ctx.consts, ctx.n_in = list(consts), len(inputs)
                ctx.save_for_backward(*inputs, *outs, *saved)
                return tuple(outs) if spec.n_out > 1 else outs[0]

            @staticmethod
            def backward(ctx, *gouts):
                t = ctx.saved_tensors
                n, m = ctx.n_in, spec.n_out
                grads = spec.bwd(ctx.consts, t[:n], t[n:n + m], t[n + m:], gouts, ctx.needs_input_grad[1:])
                return (None, *grads)

        _Eager.__name__ = f"{name}_fn"
        self.eager = _Eager

        # the real outputs must match the fake kernels' (contiguous) metadata: AOTAutograd / Inductor
        # assert sizes and strides of custom-op results
        def fwd_impl(inputs: List[Tensor], consts: List[int]) -> List[Tensor]:
            outs, saved = spec.fwd(list(consts), *inputs)
            return [t.contiguous() for t in (*outs, *saved)]

        def fwd_fake(inputs: List[Tensor], consts: List[int]) -> List[Tensor]:
            outs, saved = spec.fake(list(consts), *inputs)
            return [*outs, *saved]

        # needs[i] = 0: input i takes no gradient (ctx.needs_input_grad, as in eager mode) -- its reverse is
        # skipped and its slot is an empty placeholder, so the compiled step runs the eager step's kernels
        def bwd_impl(inputs: List[Tensor], outs: List[Tensor], saved: List[Tensor], gouts: List[Tensor],
                     consts: List[int], needs: List[int]) -> List[Tensor]:
            grads = spec.bwd(list(consts), inputs, outs, saved, gouts, [bool(n) for n in needs])
            return [x.new_empty(0) if not n else
                    g.contiguous().view(x.shape) if g is not None else torch.zeros(x.shape, dtype=x.dtype, device=x.device)
                    for g, x, n in zip(grads, inputs, needs)]

        def bwd_fake(inputs: List[Tensor], outs: List[Tensor], saved: List[Tensor], gouts: List[Tensor],
                     consts: List[int], needs: List[int]) -> List[Tensor]:
            return [x.new_empty(x.shape) if n else x.new_empty(0) for x, n in zip(inputs, needs)]

        self.fwd_op = torch.library.custom_op(f"{NS}::{name}", fwd_impl, mutates_args=())
        self.fwd_op.register_fake(fwd_fake)
        self.bwd_op = torch.library.custom_op(f"{NS}::{name}_backward", bwd_impl, mutates_args=())
        self.bwd_op.register_fake(bwd_fake)

        def setup_context(ctx, inputs, output):
            ins, consts = inputs
            ctx.consts, ctx.n_in = list(consts), len(ins)
            ctx.save_for_backward(*ins, *output)

        def backward(ctx, gouts):
            t = ctx.saved_tensors
            ins, outs = t[:ctx.n_in], t[ctx.n_in:]
            m = spec.n_out
            g = [gouts[i] if gouts[i] is not None else torch.zeros_like(outs[i]) for i in range(m)]
            needs = [int(bool(n)) for n in ctx.needs_input_grad[0]]
            grads = spec.bwd_op(list(ins), list(outs[:m]), list(outs[m:]), g, ctx.consts, needs)
            grads = [gr if n else None for gr, n in zip(grads, needs)]
            return grads, ([] if not ctx.consts else None)   # an int list is one pytree leaf

        self.fwd_op.register_autograd(backward, setup_context=setup_context)
        OPAQUE[name] = self

    def __call__(self, consts: Sequence[int], *inputs: Tensor):
        if FORCE_OPS or torch.compiler.is_compiling():
            res = self.fwd_op(list(inputs), list(consts))
            return res[0] if self.n_out == 1 else tuple(res[:self.n_out])
        return self.eager.apply(tuple(consts), *inputs)
